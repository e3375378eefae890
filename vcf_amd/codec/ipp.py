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
        if getattr(self, "lm", None) is not None:
            # the GOP loop keeps indices in HBM through the fused deadzone kernels
            raise NotImplementedError("IPP with -a LloydMax: only deadzone is on the HIP path")
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
        # the originals' PNG dumps (:641-644) run beside the coding
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=4) as dumps:
            pending = [dumps.submit(write_image, f"{self.prefix}_O_{idx:04d}.png", frames[idx])
                       for idx in range(lo * self.gop_size, min(hi * self.gop_size, len(frames)))]
            local = []
            for gi in range(lo, hi):
                g0 = gi * self.gop_size
                local.append(self._gop(frames, g0, gi, gi * (self.gop_size - 1)))
            for f in pending:
                f.result()
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
        return self.group.gather_blobs(blob)

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
    """IPP over 2D-DCT (the default --st).

    The GOP loop keeps every frame of the chain on the GPU (_gop_resident):
    the current frame is uploaded once, motion search, compensation,
    residual (or the -R mixed frame), transform + quantizer, the decoder's
    reconstruction and the next reference never leave HBM; only the indices
    (for the TIFF files), the motion field and the mode map come back, and
    their deflate + file writes run on a thread pool while the GPU carries on
    with the next frame.  A subclass that overrides encode_decode_proxy (or
    swaps the tools module) gets the frame-by-frame host loop of _IPP._gop."""

    def _code_frame(self, img, base):
        k = self.encode_indices(img)
        size = self._write_coded(base, k, img.shape)
        recon = self.decode_indices(k, img.shape)
        return recon, size

    def _write_coded(self, base, k, shape):
        with open(f"{base}_shape.bin", "wb") as f:
            f.write(struct.pack("iii", *shape))
        return self.encode_write_fn(self.compress(k), base)

    def _gop(self, frames, g0, i_idx, p0):
        if type(self).encode_decode_proxy is not _IPP.encode_decode_proxy or getattr(K, "__name__", "") != \
                "vcf_amd.ipp":
            return _IPP._gop(self, frames, g0, i_idx, p0)
        return self._gop_resident(frames, g0, i_idx, p0)

    def _gop_resident(self, frames, g0, i_idx, p0):
        import ctypes
        from concurrent.futures import ThreadPoolExecutor
        from .. import _lib
        from .. import dct as D
        from ..device import DeviceBuffer, Stream
        H, W = frames[g0].shape[:2]
        bs, n = self.block_size_ME, H * W * 3
        Hp, Wp = D.padded_shape(H, W, self.block_size)
        hb, wb = H // bs, W // bs
        s = Stream()
        cur, ref, comp, res, rec = (DeviceBuffer(n) for _ in range(5))
        dk, dmv, dgray = DeviceBuffer(Hp * Wp * 3), DeviceBuffer(max(1, hb * wb * 8)), DeviceBuffer(2 * H * W)
        dmodes = DeviceBuffer(max(1, hb * wb))
        q, flags, B = self.QSS, self.flags, self.block_size
        call, sh = _lib.call, s.handle

        def upload(img):
            a = np.ascontiguousarray(img, np.uint8)
            if a.shape != (H, W, 3):
                raise ValueError("IPP frames must share one H x W x 3 uint8 shape")
            call("vcf_memcpy_htod", cur.ptr, a.ctypes.data_as(ctypes.c_void_p), n, sh)
            s.synchronize()   # the host array may be freed after this

        def code(src, base, pool):
            """transform + quantizer of src, indices to the host for the files, decoder's frame -> rec."""
            D.encode_device(src, 1, H, W, q, flags, out=dk, stream=s, block_size=B)
            k = np.empty((Hp, Wp, 3), np.uint8)
            call("vcf_memcpy_dtoh", k.ctypes.data_as(ctypes.c_void_p), dk.ptr, k.nbytes, sh)
            D.decode_device(dk, 1, H, W, q, flags, out=rec, stream=s, block_size=B)
            s.synchronize()
            return pool.submit(self._write_coded, base, k, (H, W, 3))

        P, mvs = [], []
        try:
            with ThreadPoolExecutor(max_workers=8) as pool:
                upload(frames[g0])
                fut_I = code(cur, f"{self.prefix}_I_{i_idx}_enc", pool)
                call("vcf_memcpy_dtod", ref.ptr, rec.ptr, n, sh)
                futs = []
                for p in range(1, min(self.gop_size, len(frames) - g0)):
                    upload(frames[g0 + p])
                    call("vcf_ipp_block_match", ref.ptr, cur.ptr, H, W, bs, int(self.search_range),
                         int(bool(self.use_fast)), dmv.ptr, dgray.ptr, sh)
                    call("vcf_ipp_motion_compensate", ref.ptr, dmv.ptr, H, W, bs, comp.ptr, sh)
                    mv = np.zeros((hb, wb, 2), np.float32)
                    if mv.size:
                        call("vcf_memcpy_dtoh", mv.ctypes.data_as(ctypes.c_void_p), dmv.ptr, mv.nbytes, sh)
                    if self.rdo_lambda > 0:
                        # :441-536: per-block I/P decision, the mixed-mode frame, its reconstruction
                        modes = np.zeros((hb, wb), np.uint8)
                        if modes.size:
                            call("vcf_ipp_rdo_modes", cur.ptr, comp.ptr, H, W, bs, int(q), float(self.rdo_lambda),
                                 dmodes.ptr, None, sh)
                            call("vcf_memcpy_dtoh", modes.ctypes.data_as(ctypes.c_void_p), dmodes.ptr, modes.nbytes,
                                 sh)
                        call("vcf_ipp_rdo_residual", cur.ptr, comp.ptr, dmodes.ptr, H, W, bs, res.ptr, sh)
                        futs.append(code(res, f"{self.prefix}_P_{p0 + p - 1}_enc", pool))
                        call("vcf_ipp_rdo_reconstruct", comp.ptr, rec.ptr, dmodes.ptr, H, W, bs, ref.ptr, sh)
                        n_i = int(modes.sum())
                        logging.info(f"  RDO (λ={self.rdo_lambda}): {n_i}/{modes.size} I-blocks, "
                                     f"{modes.size - n_i}/{modes.size} P-blocks")
                        mvs.append({"mv": mv, "modes": modes})
                    else:
                        call("vcf_ipp_residual", cur.ptr, comp.ptr, n, res.ptr, sh)
                        futs.append(code(res, f"{self.prefix}_P_{p0 + p - 1}_enc", pool))
                        call("vcf_ipp_reconstruct", comp.ptr, rec.ptr, n, ref.ptr, sh)
                        mvs.append(mv)
                s.synchronize()
                I = {"bits": fut_I.result(), "idx": g0}
                P = [{"bits": f.result()} for f in futs]
        finally:
            for b in (cur, ref, comp, res, rec, dk, dmv, dgray, dmodes):
                b.free()
            s.close()
        return I, P, mvs, []

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
