"""III video coding: the drop-in for src/III.py (CoDec over video_coding.CoDec).

A 2D image codec (-T, default 2D-DCT) runs on every frame of a sequence,
with the reference's file naming (III.py:73-118,120-144;
video_coding.py:22-27): frames are read from /tmp/original_%04d.png, coded
into /tmp/encoded_%04d{.tif,_shape.bin}, decoded into /tmp/decoded_%04d.png.

The reference's encode() demuxes a video with PyAV into those PNGs and then
stops (the per-frame encode_fn call is commented out, III.py:100-104); here
encode() extracts the frames the same way when the input is a video and PyAV
is importable (it is not in this image), and then codes every frame, which
is what the decode side expects.  The input may also be a printf pattern
('/tmp/original_%04d.png') or a directory of PNGs.

Frames are sharded over the ranks of the job (one process per GPU, see
shard.py); each rank codes its contiguous chunk in batches through the
transform codec's encode_fns/decode_fns (one GPU launch per batch), and the
per-frame sizes are all-gathered so rank 0 can report the totals.
"""
from __future__ import annotations

import glob
import logging
import os

from . import shard

ENCODE_OUTPUT_PREFIX = "/tmp/encoded"     # video_coding.py:23
DECODE_OUTPUT_PREFIX = "/tmp/decoded"     # :25
ORIGINAL_PATTERN = "/tmp/original_%04d.png"


def transform_codec(args):
    name = getattr(args, "transform", "2D-DCT")
    if name == "2D-DCT":
        from .dct2d import CoDec
        return CoDec(args)
    if name == "2D-DWT":
        from .dwt2d import CoDec
        return CoDec(args)
    raise NotImplementedError(f"transform {name!r}: 2D-DCT and 2D-DWT are on the HIP path")


def _frame_inputs(original: str, n: int):
    if "%" in original:
        return [original % i for i in range(n)]
    if os.path.isdir(original):
        files = sorted(glob.glob(os.path.join(original, "*.png")))
        return files[:n]
    if original.lower().endswith(".png"):
        return [original][:n]
    try:
        import av  # noqa: F401  (PyAV: absent in this image)
    except ImportError as e:
        raise NotImplementedError(f"{original}: video demux needs PyAV, which is not installed; "
                                  f"pass a frame pattern like {ORIGINAL_PATTERN}") from e
    return _extract_frames(original, n)


def _extract_frames(fn: str, n: int):
    """III.py:73-112: demux with PyAV, write /tmp/original_%04d.png."""
    import av
    import numpy as np
    from .eic import write_image
    out = []
    with av.open(fn) as container:
        for frame in container.decode(video=0):
            img_fn = ORIGINAL_PATTERN % len(out)
            write_image(img_fn, np.array(frame.to_image().convert("RGB")))
            out.append(img_fn)
            if len(out) >= n:
                break
    return out


class CoDec:
    """III.CoDec (III.py:50-144) with frame sharding."""

    def __init__(self, args, codec=None, group=None, batch: int = 64,
                 encode_prefix: str = ENCODE_OUTPUT_PREFIX, decode_prefix: str = DECODE_OUTPUT_PREFIX):
        self.args = args
        self.encoding = args.subparser_name == "encode"
        # a multi-rank Group selects this rank's GPU (local rank) before any codec work
        self.group = group if group is not None else shard.Group()
        self.transform_codec = codec if codec is not None else transform_codec(args)
        self.batch = batch
        self.encode_prefix = encode_prefix
        self.decode_prefix = decode_prefix
        self.total_input_size = 0
        self.total_output_size = 0
        self.sizes = None
        logging.info(f"Using {getattr(args, 'transform', '2D-DCT')} codec")

    def bye(self):
        return None

    def _n(self):
        return int(self.args.number_of_frames)

    def encode(self):
        g = self.group
        n_req = self._n()
        inputs = _frame_inputs(str(self.args.original), n_req)
        n = len(inputs)
        lo, hi = shard.frame_range(n, g.rank, g.world)
        pairs = [(inputs[i], f"{self.encode_prefix}_%04d" % i) for i in range(lo, hi)]
        local = self.transform_codec.encode_fns(pairs, batch=self.batch) if pairs else []
        self.sizes = g.all_gather_sizes(n, local)
        self.N_frames = n
        self.total_output_size = int(self.sizes.sum())
        logging.info(f"III encode: {n} frames, {self.total_output_size} bytes (rank {g.rank}/{g.world})")
        return self.total_output_size

    def decode(self):
        g = self.group
        n = self._n()
        lo, hi = shard.frame_range(n, g.rank, g.world)
        pairs = [(f"{self.encode_prefix}_%04d" % i, f"{self.decode_prefix}_%04d.png" % i)
                 for i in range(lo, hi)]
        local = self.transform_codec.decode_fns(pairs, batch=self.batch) if pairs else []
        self.sizes = g.all_gather_sizes(n, local)
        self.total_output_size = int(self.sizes.sum())
        return self.total_output_size

    def gather_codestreams(self):
        """Rank 0: every frame's .tif bytes in frame order (§8(e) exchange step)."""
        g = self.group
        n = len(self.sizes)
        lo, hi = shard.frame_range(n, g.rank, g.world)
        ext = getattr(self.transform_codec, "file_extension", ".tif")
        local = [open(f"{self.encode_prefix}_%04d" % i + ext, "rb").read() for i in range(lo, hi)]
        return g.gather_payloads(n, local, self.sizes)
