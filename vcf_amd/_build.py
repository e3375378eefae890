"""Build recipe for libvcf_amd.so (hipcc, gfx950) -- used by __graft_entry__.build().

The library is built in-tree (vcf_amd/libvcf_amd.so) so it travels to the GPU
box with the repository snapshot.  A second, experimental library
(vcf_amd/libvcf_amd_ab.so, include/vcf_amd_ab.h) holds the A/B kernel
variants the product defaults were measured against (csrc/ab/); the A/B
scripts and the cross-check tests load it, the product path never does.
"""
from __future__ import annotations

import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libvcf_amd.so")
AB_LIB = os.path.join(PKG, "libvcf_amd_ab.so")
# the A/B archive's own sources, linked with these product objects
AB_SOURCES = ["ab/vcf_dct_dz_ab.hip", "ab/vcf_dwt_ab.hip", "ab/vcf_inflate_wincheck.hip"]
AB_LINK = ["vcf_runtime.hip", "vcf_dct_any.hip"]
SOURCES = ["vcf_runtime.hip", "vcf_dct_dz.hip", "vcf_dct_any.hip", "vcf_quant.hip", "vcf_dwt.hip", "vcf_cbaac.cpp",
           "vcf_cbahc.cpp", "vcf_ipp.hip", "vcf_ipp_rdo.hip",
           "vcf_png.cpp", "vcf_comm.cpp", "vcf_cbaac_gpu.hip", "vcf_plugins.hip", "vcf_deflate.hip",
           "vcf_inflate.hip"]
HEADERS = ["vcf_dct8.h", "vcf_dct_block.h", "vcf_internal.h", "vcf_wavelets.h", "vcf_pocketfft.h", "vcf_pocketfft_tables.h",
           "vcf_pocketfft_rt.h", "vcf_pocketfft_blue.h", "vcf_sincos.h", "vcf_pipeline.h", "vcf_dwt_band.h", "vcf_idwt_line.h", "vcf_idwt_band21.h",
           "vcf_dwt_lift.h",
           "vcf_deflate.h"]
OBJDIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("VCF_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build libvcf_amd.so)")


def deps_mtime(src: str) -> float:
    """Newest mtime of a source and the local headers it includes (transitively)."""
    seen, todo, newest = set(), [os.path.join(CSRC, src)], 0.0
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(f):
            continue
        seen.add(f)
        newest = max(newest, os.path.getmtime(f))
        for name in local_includes(f):
            for d in (CSRC, os.path.join(ROOT, "include")):
                if os.path.exists(os.path.join(d, name)):
                    todo.append(os.path.join(d, name))
                    break
    return newest


def local_includes(path: str) -> list:
    """The `#include "..."` names of one file."""
    out = []
    for line in open(path, errors="replace"):
        line = line.strip()
        if line.startswith("#include \""):
            out.append(line.split('"')[1])
    return out


def needs_rebuild() -> bool:
    """True when either library is missing or older than any source or any
    header a source includes, directly or transitively (the same scan
    build() uses per object)."""
    if not os.path.exists(LIB) or not os.path.exists(AB_LIB):
        return True
    t = min(os.path.getmtime(LIB), os.path.getmtime(AB_LIB))
    deps = [os.path.join(CSRC, s) for s in HEADERS]
    deps += [os.path.join(ROOT, "include", h) for h in ("vcf_amd.h", "vcf_amd_ab.h")]
    newest = max([deps_mtime(s) for s in SOURCES + AB_SOURCES] + [os.path.getmtime(d) for d in deps if os.path.exists(d)])
    return newest > t


def _flags():
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17",
            # bit-exactness: pocketfft's separate multiply and add must not fuse
            "-ffp-contract=off",
            "-fPIC", "-Wall",
            "-I", os.path.join(ROOT, "include"), "-I", CSRC]


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile each translation unit to an object (in parallel), then link."""
    if not force and not needs_rebuild():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(OBJDIR, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        path = os.path.join(CSRC, src)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > deps_mtime(src):
            return obj
        cmd = [hipcc(), *_flags(), "-c", path, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        return obj

    everything = SOURCES + AB_SOURCES
    jobs = max(1, min(len(everything), int(os.environ.get("MAX_JOBS", "8")), os.cpu_count() or 1))
    with ThreadPoolExecutor(jobs) as ex:
        objs = dict(zip(everything, ex.map(compile_one, everything)))

    def link(lib, srcs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *[objs[x] for x in srcs], "-lz", "-ldl",
               "-o", lib + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(lib + ".tmp", lib)

    link(LIB, SOURCES)
    link(AB_LIB, AB_SOURCES + AB_LINK)
    return LIB


if __name__ == "__main__":
    build(force=True, verbose=True)
