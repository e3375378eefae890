#!/usr/bin/env python3
"""Tiled CBAAC kernel timing, one segment per wave (variant 1) vs one per
lane (variant 2), order 0, prior-seeded (-c TCBAACP): one 1080p frame, and
batches of 1080p frames coded in one launch (throughput).  One JSON line each.
usage: bench_tcbaac_lane.py [frames,frames,...] [seg_len,...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from vcf_amd.synthetic import synth_frame
    import vcf_amd.dct as D
    from vcf_amd import _lib as L
    from vcf_amd import tcbaac as T
    from vcf_amd.device import DeviceBuffer, Event, Stream, set_device
    set_device(0)
    batches = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16").split(",")]
    seg_lens = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "32768,24576").split(",")]
    ks = [D.encode(synth_frame(1080, 1920, s), 32).ravel() for s in range(4)]
    cases = [("1x1080p", ks[0], 5)] + [(f"{b}x1080p", np.concatenate([ks[f % 4] for f in range(b)]), 2)
                                       for b in batches]
    lib = L.lib()
    st = Stream()

    def timed(fn, reps):
        fn()
        st.synchronize()
        e0, e1 = Event(), Event()
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        st.synchronize()
        return e0.elapsed_ms(e1) / reps

    for seg_len in seg_lens:
        for variant in (1, 2):
            L.call("vcf_cbaac_tiled_set_variant", variant)
            for name, sym, reps in cases:
                n = sym.size
                coder = T.TiledCoder(0, seg_len, stream=st, prior=True)
                sizes, payload = coder.encode(sym)
                prior = coder.last_prior
                dsym = DeviceBuffer.from_array(sym, st)
                ws = DeviceBuffer(int(lib.vcf_cbaac_tiled_workspace(n, seg_len)))
                cap = int(lib.vcf_cbaac_tiled_bound(n, seg_len))
                out, sb = DeviceBuffer(cap), DeviceBuffer(8 * (len(sizes) + 1))
                pr = DeviceBuffer.from_array(prior, st)
                enc = timed(lambda: L.call("vcf_cbaac_tiled_encode_prior", dsym.ptr, n, 0, pr.ptr, seg_len, out.ptr,
                                           cap, sb.ptr, ws.ptr, st.handle), reps)
                offs = DeviceBuffer.from_array(np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64), st)
                src = DeviceBuffer.from_array(np.frombuffer(payload, np.uint8), st)
                dec_out = DeviceBuffer(n)
                dec = timed(lambda: L.call("vcf_cbaac_tiled_decode_prior", src.ptr, offs.ptr, n, 0, pr.ptr, seg_len,
                                           dec_out.ptr, st.handle), reps)
                back = np.empty(n, np.uint8)
                dec_out.download(back)
                print(json.dumps(dict(case="tcbaacp", variant=["auto", "wave", "lane"][variant], frames=name, seg_len=seg_len,
                                      segments=len(sizes), symbols=n, bytes=len(payload),
                                      encode_ms=round(enc, 3), decode_ms=round(dec, 3),
                                      encode_Gsym_s=round(n / enc / 1e6, 3), decode_Gsym_s=round(n / dec / 1e6, 3),
                                      round_trip=bool(np.array_equal(back, sym)))), flush=True)
    L.call("vcf_cbaac_tiled_set_variant", 0)


if __name__ == "__main__":
    main()
