"""IPP hybrid video coding: the drop-in for src/IPP_DCT.py (IPP + CoDec).

Each GOP is an I-frame coded by the spatial codec (--st: 2D-DCT, the
default, or 2D-DWT -- the reference subclasses whichever module --st names,
IPP_DCT.py:45-87; here codec_class(st) picks CoDec or CoDecDWT)
followed by P-frames: block matching against the previous reconstruction,
motion compensation, the residual shifted by 128 and clipped, coded by the
same spatial codec, and the reconstruction clip(pred + rec - 128)
(IPP_DCT.py:397-575).  Files are the reference's: {prefix}_O_%04d.png
(originals), {prefix}_{I,P}_{n}_enc.tif + _shape.bin, {prefix}_mv.npz,
{prefix}_meta.json; decode writes {out}_%04d.png.

Block matching, compensation, residual and reconstruction run on the GPU
(vcf_amd/csrc/vcf_ipp.hip); the spatial codec is the 2D-DCT CoDec (GPU).
encode_decode_proxy (:595-626) round-trips through temporary PNG files in
the reference; here the coded frame is decoded from the same code-stream in
memory (PNG is lossless, so the reconstruction is identical).

GOPs are independent, so they shard over ranks (one process per GPU); the
per-frame sizes and motion fields are gathered on rank 0, which writes the
metadata (at most ceil(N/G) ranks are busy).
-R/--rdo_lambda > 0 runs the block-level mode decision on the GPU
(vcf_amd/csrc/vcf_ipp_rdo.hip: rdo_block_decision :290-342 per block, the
mixed-mode frame :489-505 and its reconstruction :512-526); the motion file
then also carries each P frame's mode map, like the reference's
{"mv", "modes"} entries, and the decoder reconstructs mode by mode
(:770-790).
"""
from __future__ import annotations

import glob
import io
import json
import logging
import os
import struct

import numpy as np

from .. import ipp as K
from . import shard
from .dct2d import CoDec as DCTCoDec
from .dwt2d import CoDec as DWTCoDec
from .eic import read_image, write_image

_TMP_DIR = "/tmp"   # os.path.join(_SCRIPT_DIR, "/tmp") == "/tmp" (IPP_DCT.py:20)


def resolve_prefix(prefix: str) -> str:
    """IPP_DCT.py:132-142."""
    if prefix.startswith("./"):
        return os.path.join(_TMP_DIR, prefix[2:])
    if not os.path.isabs(prefix):
        return os.path.join(_TMP_DIR, prefix)
    return prefix


def _ensure_dir(prefix: str):
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)


def read_frames(src: str, n: int):
    """The encoder's input: a video (needs PyAV, absent here), a printf
    pattern of PNGs, a directory of PNGs or an .npy (N x H x W x 3)."""
    if src.endswith(".npy"):
        return list(np.load(src, allow_pickle=False)[:n])
    if "%" in src:
        files = [src % i for i in range(n)]
    elif os.path.isdir(src):
        files = sorted(glob.glob(os.path.join(src, "*.png")))[:n]
    else:
        try:
            import av
        except ImportError as e:
            raise NotImplementedError(f"{src}: video demux needs PyAV, which is not installed; pass a PNG "
                                      f"pattern, a directory of PNGs or an .npy of frames") from e
        frames = []
        with av.open(src) as c:
            for fr in c.decode(video=0):
                frames.append(np.array(fr.to_image().convert("RGB")))
                if len(frames) >= n:
                    break
        return frames
    return [read_image(f)[0] for f in files]


class _IPP:
    """IPP_DCT.CoDec (:578-720) over a spatial codec base class (the MRO's next)."""

    def __init__(self, args, group=None):
        super().__init__(args)
        self.gop_size = getattr(args, "gop_size", 10) or 10
        self.block_size_ME = getattr(args, "block_size_ME", 16) or 16
        self.search_range = getattr(args, "search_range", 8)
        if self.search_range is None:
            self.search_range = 8
        self.use_fast = bool(getattr(args, "fast", False))
        self.rdo_lambda = float(getattr(args, "rdo_lambda", 0.0) or 0.0)
        self.prefix = resolve_prefix(args.output) if getattr(args, "output", None) else None
        self.group = group if group is not None else shard.Group()

    def bye(self):
        if getattr(self, "N_frames", 0) and hasattr(self, "total_bits"):
            bpp = self.total_bits / (self.N_frames * self.width * self.height)
            logging.info(f"Output bit-rate = {bpp:.4f} bits/pixel")

    # IPP_DCT.py:595-626: encode_fn to the frame's files, decode_fn back (in memory)
    def encode_decode_proxy(self, img, frame_type, seq_idx):
        return self._code_frame(img, f"{self.prefix}_{frame_type}_{seq_idx}_enc")

    def _gop(self, frames, g0, i_idx, p0):
        """One GOP: I-frame then P-frames (IPP.temporal_filter :397-575)."""
        bs = self.block_size_ME
        recon_I, bits_I = self.encode_decode_proxy(frames[g0], "I", i_idx)
        I = {"bits": bits_I, "idx": g0}
        P, mvs, recon = [], [], [recon_I]
        ref = recon_I
        for p in range(1, min(self.gop_size, len(frames) - g0)):
            cur = frames[g0 + p]
            mv = K.block_matching(ref, cur, bs, self.search_range, self.use_fast)
            comp = K.motion_compensate(ref, mv, bs)
            if self.rdo_lambda > 0:
                # :441-536: per-block I/P decision, the mixed-mode frame, its reconstruction
                modes = K.rdo_modes(cur, comp, bs, self.QSS, self.rdo_lambda)
                res = K.rdo_residual(cur, comp, modes, bs)
                rec_res, bits_P = self.encode_decode_proxy(res, "P", p0 + p - 1)
                ref = K.rdo_reconstruct(comp, rec_res, modes, bs)
                n_i = int(modes.sum())
                logging.info(f"  RDO (λ={self.rdo_lambda}): {n_i}/{modes.size} I-blocks, "
                             f"{modes.size - n_i}/{modes.size} P-blocks")
                mvs.append({"mv": mv, "modes": modes})
            else:
                res = K.residual(cur, comp)
                rec_res, bits_P = self.encode_decode_proxy(res, "P", p0 + p - 1)
                ref = K.reconstruct(comp, rec_res)
                mvs.append(mv)
            P.append({"bits": bits_P})
            recon.append(ref)
        return I, P, mvs, recon

    def encode(self):
        g = self.group
        frames = read_frames(str(self.args.input), int(self.args.number_of_frames))
        if len(frames) < 2:
            raise ValueError("Need at least 2 frames for IPP structure")
        self.N_frames = len(frames)
        self.height, self.width = frames[0].shape[:2]
        _ensure_dir(self.prefix)
        n_gops = (len(frames) + self.gop_size - 1) // self.gop_size
        lo, hi = shard.frame_range(n_gops, g.rank, g.world)
        for idx in range(lo * self.gop_size, min(hi * self.gop_size, len(frames))):
            write_image(f"{self.prefix}_O_{idx:04d}.png", frames[idx])
        local = []
        for gi in range(lo, hi):
            g0 = gi * self.gop_size
            local.append(self._gop(frames, g0, gi, gi * (self.gop_size - 1)))
        # gather per-GOP results on rank 0 (sizes as JSON, motion fields as bytes)
        blob = json.dumps([[I, P] for I, P, _, _ in local]).encode()
        rdo = self.rdo_lambda > 0
        mv_of = (lambda m: m["mv"]) if rdo else (lambda m: m)
        mvbytes = b"".join(mv_of(m).astype(np.float32).tobytes() for _, _, mvs, _ in local for m in mvs)
        infos = self._gather(blob)
        mvs_all = self._gather(mvbytes)
        if rdo:
            modes_all = self._gather(b"".join(m["modes"].tobytes() for _, _, mvs, _ in local for m in mvs))
        if g.rank != 0:
            return None
        I_infos, P_infos = [], []
        for b in infos:
            for I, P in json.loads(b):
                I_infos.append(I)
                P_infos.extend(P)
        hb, wb = self.height // self.block_size_ME, self.width // self.block_size_ME
        mv = np.frombuffer(b"".join(mvs_all), np.float32).reshape(len(P_infos), hb, wb, 2)
        mv_path = f"{self.prefix}_mv.npz"
        if rdo:
            # the reference's entries are {"mv": field, "modes": map} (:529)
            modes = np.frombuffer(b"".join(modes_all), np.uint8).reshape(len(P_infos), hb, wb)
            obj = np.empty(len(P_infos), dtype=object)
            for i in range(len(P_infos)):
                obj[i] = {"mv": mv[i], "modes": modes[i]}
            np.savez_compressed(mv_path, mv=obj, mv_f32=mv, modes_u8=modes)
        else:
            obj = np.empty(len(P_infos), dtype=object)
            for i in range(len(P_infos)):
                obj[i] = mv[i]
            np.savez_compressed(mv_path, mv=np.array(list(obj), dtype=object), mv_f32=mv)
        total_bits = sum(i["bits"] for i in I_infos) + sum(p["bits"] for p in P_infos)
        total_bits += os.path.getsize(mv_path) * 8
        self.total_bits = total_bits
        meta = {"n_frames": self.N_frames, "width": self.width, "height": self.height, "gop_size": self.gop_size,
                "total_bits": total_bits, "I_info": I_infos, "P_info": P_infos,
                "mv_file": f"{os.path.basename(self.prefix)}_mv.npz", "base_prefix": os.path.basename(self.prefix)}
        with open(f"{self.prefix}_meta.json", "w") as f:
            json.dump(meta, f, indent=4)
        return total_bits

    def _gather(self, blob: bytes):
        """Rank 0: every rank's blob in rank order (item r belongs to rank r)."""
        g = self.group
        if g.dist is None:
            return [blob]
        sizes = g.all_gather_sizes(g.world, [len(blob)])
        return g.gather_payloads(g.world, [blob], sizes)

    def decode(self):
        in_prefix = resolve_prefix(self.args.input)
        with open(f"{in_prefix}_meta.json") as f:
            meta = json.load(f)
        mv_path = f"{os.path.dirname(in_prefix)}/{meta['mv_file']}"
        with np.load(mv_path, allow_pickle=False) as z:
            if "mv_f32" not in z.files:
                raise NotImplementedError(f"{mv_path}: motion fields stored only as a pickled object array "
                                          "(written by the reference); re-encode or convert to 'mv_f32'")
            mvs = z["mv_f32"]
            modes = z["modes_u8"] if "modes_u8" in z.files else None
        out_prefix = resolve_prefix(self.args.output)
        _ensure_dir(out_prefix)
        gop, N = meta["gop_size"], meta["n_frames"]
        bs = self.block_size_ME
        recon, p_idx = [], 0
        for i_idx, g0 in enumerate(range(0, N, gop)):
            if i_idx >= len(meta["I_info"]):
                break
            ref = self._decode_frame(f"{in_prefix}_I_{i_idx}_enc")
            recon.append(ref)
            for p in range(1, min(gop, N - g0)):
                rec_res = self._decode_frame(f"{in_prefix}_P_{p_idx}_enc")
                pred = K.motion_compensate(ref, mvs[p_idx], bs)
                if modes is not None:   # RDO was used: mode-aware reconstruction (:770-790)
                    ref = K.rdo_reconstruct(pred, rec_res, modes[p_idx], bs)
                else:
                    ref = K.reconstruct(pred, rec_res)
                recon.append(ref)
                p_idx += 1
        for idx, img in enumerate(recon):
            write_image(f"{out_prefix}_{idx:04d}.png", img)
        logging.warning("decoded MP4 not written (needs PyAV/imageio, not installed); PNG frames are")
        self.recon = recon
        return len(recon)



class CoDec(_IPP, DCTCoDec):
    """IPP over 2D-DCT (the default --st)."""

    def _code_frame(self, img, base):
        k = self.encode_indices(img)
        with open(f"{base}_shape.bin", "wb") as f:
            f.write(struct.pack("iii", *img.shape))
        cs = self.compress(k)
        data = cs.getvalue()
        size = self.encode_write_fn(io.BytesIO(data), base)
        recon = self.decode_indices(self.decompress(data), img.shape)
        return recon, size

    def _decode_frame(self, base):
        data = self.decode_read_fn(base)
        with open(f"{base}_shape.bin", "rb") as f:
            shape = struct.unpack("iii", f.read(12))
        return self.decode_indices(self.decompress(data), shape)


class CoDecDWT(_IPP, DWTCoDec):
    """IPP over 2D-DWT (--st 2D-DWT): each frame's 3l+1 subband TIFFs
    ({base}_LL_l.tif, {base}_{LH,HL,HH}_r.tif, 2D-DWT.py:162-200).  The
    reconstruction is waverec2's 2*ceil(H/2) x 2*ceil(W/2), as in the
    reference (whose IPP loop therefore needs even frame sides)."""

    def _code_frame(self, img, base):
        from .. import dwt as DW
        if img.ndim != 3 or img.shape[2] != 3 or img.dtype != np.uint8:
            raise ValueError("Input image must be a 3D array (height, width, channels).")
        sb = DW.encode(img, self.wavelet, self.levels, self.QSS)[0]
        size = self.write_decom_fn(sb, base)
        H, W = self._geometry(sb)
        return DW.decode(sb, H, W, self.wavelet, self.levels, self.QSS), size

    def _decode_frame(self, base):
        from .. import dwt as DW
        sb = self.read_decom_fn(base)
        H, W = self._geometry(sb)
        return DW.decode(sb, H, W, self.wavelet, self.levels, self.QSS)


def codec_class(space_transform: str = "2D-DCT"):
    """The IPP codec class over the spatial codec --st names (IPP_DCT.py:45-87)."""
    if space_transform == "2D-DCT":
        return CoDec
    if space_transform == "2D-DWT":
        return CoDecDWT
    raise NotImplementedError(f"--st {space_transform}: 2D-DCT and 2D-DWT are on the HIP path")
