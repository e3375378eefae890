"""Build recipe for libvcf_amd.so (hipcc, gfx950) -- used by __graft_entry__.build().

The library is built in-tree (vcf_amd/libvcf_amd.so) so it travels to the GPU
box with the repository snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libvcf_amd.so")
SOURCES = ["vcf_runtime.hip", "vcf_dct_dz.hip", "vcf_dct_any.hip", "vcf_quant.hip", "vcf_dwt.hip", "vcf_cbaac.cpp",
           "vcf_cbahc.cpp", "vcf_ipp.hip", "vcf_ipp_rdo.hip",
           "vcf_png.cpp", "vcf_comm.cpp", "vcf_cbaac_gpu.hip", "vcf_plugins.hip"]
HEADERS = ["vcf_dct8.h", "vcf_dct_block.h", "vcf_internal.h", "vcf_wavelets.h", "vcf_pocketfft.h", "vcf_pocketfft_tables.h",
           "vcf_pocketfft_rt.h", "vcf_pipeline.h", "vcf_dwt_band.h", "vcf_idwt_line.h"]
OBJDIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("VCF_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build libvcf_amd.so)")


def needs_rebuild() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "vcf_amd.h"))
    return any(os.path.getmtime(d) > t for d in deps)


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

    def deps_mtime(src):
        """Newest mtime of a source and the local headers it includes (transitively)."""
        seen, todo, newest = set(), [os.path.join(CSRC, src)], 0.0
        while todo:
            f = todo.pop()
            if f in seen or not os.path.exists(f):
                continue
            seen.add(f)
            newest = max(newest, os.path.getmtime(f))
            for line in open(f, errors="replace"):
                line = line.strip()
                if line.startswith("#include \""):
                    name = line.split('"')[1]
                    for d in (CSRC, os.path.join(ROOT, "include")):
                        if os.path.exists(os.path.join(d, name)):
                            todo.append(os.path.join(d, name))
                            break
        return newest

    def compile_one(src):
        obj = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
        path = os.path.join(CSRC, src)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > deps_mtime(src):
            return obj
        cmd = [hipcc(), *_flags(), "-c", path, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "8")), os.cpu_count() or 1))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-lz", "-ldl", "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force=True, verbose=True)
