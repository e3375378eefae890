"""Per-phase clock totals of the GPU deflate's parse kernels and K1 (zlib_sort_kernel) (diagnostic build
scripts/libvcf_zprof.so, VCF_ZLIB_PROF): one vcf_zlib_strips call over the C4
workload, then the counters.  Prints one JSON line."""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vcf_amd.synthetic import synth_frame, c4_frame
from vcf_amd import _lib as L, dct
from vcf_amd.codec.tiff import strip_layout
from vcf_amd.device import DeviceBuffer, Stream, Event
P = ctypes.CDLL(os.path.join(ROOT, "scripts", "debug", os.environ.get("ZPROF_LIB", "libvcf_zprof.so")))
P.vcf_zlib_strips.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                              ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
P.vcf_zlib_workspace.restype = ctypes.c_int64
P.vcf_zlib_workspace.argtypes = [ctypes.c_int64]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H, W = 1080, 1920
bases = [synth_frame(H, W, seed=100 + s) for s in range(4)]
frames = np.concatenate([dct.encode(np.stack([c4_frame(bases, i) for i in range(f, min(n, f + 16))]), Q=32)
                         for f in range(0, n, 16)])
flat = np.ascontiguousarray(frames.reshape(n, -1))
fb = flat.shape[1]; _, _, sb = strip_layout(frames.shape[1:], 1)
spf = int(L.lib().vcf_zlib_strip_count(fb, sb)); total = spf * n; slot = int(L.lib().vcf_zlib_bound(sb))
d = DeviceBuffer.from_array(flat); out = DeviceBuffer(total * slot); sizes = DeviceBuffer(total * 4)
ws = DeviceBuffer(int(P.vcf_zlib_workspace(total))); st = Stream()
buf = (ctypes.c_ulonglong * 48)()
for rep in range(2):
    P.vcf_zlib_prof_read(buf, 1)
    e0, e1 = Event(), Event()
    e0.record(st)
    assert P.vcf_zlib_strips(d.ptr, n, fb, sb, 6, out.ptr, slot, sizes.ptr, ws.ptr, st.handle) == 0
    e1.record(st); st.synchronize()
    P.vcf_zlib_prof_read(buf, 0)
v = list(buf)
ns = max(1, v[6])
print(json.dumps({"frames": n, "strips": total, "ms": round(e0.elapsed_ms(e1), 2), "lazy_strips": v[6],
                  "lazy_cycles_per_strip": v[0] // ns, "longest_cycles_per_strip": v[1] // ns,
                  "flush_cycles_per_strip": v[2] // ns, "longest_calls_per_strip": v[3] / ns,
                  "chain_rounds_per_strip": v[4] / ns, "shifts_per_strip": v[5] / ns,
                  "cycles_per_longest": v[1] // max(1, v[3]),
                  "k3_cycles_per_strip": v[7] // max(1, total - v[6]),
                  "head_cycles_per_longest": v[8] // max(1, v[3]), "lcp_steps_per_round": v[9] / max(1, v[4]),
                  "scan_end_passes_per_round": v[10] / max(1, v[4]), "prefetch_served": v[11] / max(1, v[3]),
                  "cand_wait_cycles_per_longest": v[12] // max(1, v[3]),
                  "round_cycles_to_chain_ballot": v[13] // max(1, v[4]), "round_cycles_to_lengths": v[14] // max(1, v[4]),
                  "round_cycles_rest": v[15] // max(1, v[4]),
                  "head_hit_frac": v[16] / max(1, v[3]), "far_round_frac": v[17] / max(1, v[4]),
                  "far_lcp_lanes_per_round": v[18] / max(1, v[4]), "far_final_compare_per_call": v[19] / max(1, v[3]),
                  "far_head_frac": v[20] / max(1, v[3]), "no_match_frac": v[21] / max(1, v[3]),
                  "sort_workgroups": v[47], **{f"sort_{nm}_cycles": v[40 + i] // max(1, v[47]) for i, nm in enumerate(
                      ("count1", "scan1", "place1", "scan2", "place2", "firsts"))},
                  "lib": os.environ.get("ZPROF_LIB", "libvcf_zprof.so")}), flush=True)
