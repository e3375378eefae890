"""2D-DCT image codec: the drop-in for src/2D-DCT.py's CoDec.

Same constructor (an argparse Namespace, see parser.py), same methods and
return values (encode_fn/decode_fn -> bytes written; encode/decode with the
reference's hard-wired default paths; bye), same files ({out}.tif holding
the k + 128 indices in subband layout, {out}_shape.bin = struct 'iii').  The
span between reading the image and handing the indices to the entropy codec
-- 2D-DCT.py:276-361 encode, :399-466 decode -- runs on the GPU through
libvcf_amd.so (vcf_dct_dz_encode / vcf_dct_dz_decode); there is no CPU
implementation of it in the product.

-B takes every block size the HIP path has a transform for (every B <= 4096,
vcf_dct_block_size_supported: pocketfft's rfftp plans and its Bluestein
lengths, the first of which is 191), -L runs optimize_block_size
(2D-DCT.py:533-579) with the GPU doing each candidate's analysis/synthesis.
-t YCrCb runs exactly as -t YCoCg: 2D-DCT.py binds from_RGB/to_RGB from
color_transforms.YCoCg at import (:22-23) and -t only picks the base class
(:54-56), whose encode/decode it overrides.  -a LloydMax (LloydMax.py) sets
the offset to 0 (:106-109): the GPU hands the float32 coefficients to the
Lloyd-Max quantizer (histogram, design, encoder on the GPU,
codec/quantizers.py) and decodes from its int16 output.  Options the HIP
path does not implement raise NotImplementedError when the codec is
constructed (block sizes above 4096, other colour transforms, quantizers
other than deadzone and LloydMax, filters other than no_filter, -L with
LloydMax); entropy codecs come from ENTROPY_CODECS.
"""
from __future__ import annotations

import io
import logging
import struct
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .. import dct as D
from ..device import DeviceBuffer
from .eic import CoDec as EICCoDec
from .quantizers import LloydMaxQuantizer
from .tiff import TIFFCodec


def _cbaac(args=None):
    from ..cbaac import CBAACCodec
    return CBAACCodec(getattr(args, "order", 0) if args is not None else 0)


def _cbahc(args=None):
    from ..cbahc import CBAHCCodec
    return CBAHCCodec(getattr(args, "order", 0) if args is not None else 0)


def _tcbaac(args=None):
    from ..tcbaac import DEFAULT_SEG, TiledCBAACCodec
    return TiledCBAACCodec(getattr(args, "order", 0) if args is not None else 0,
                           getattr(args, "segment_symbols", DEFAULT_SEG) if args is not None else DEFAULT_SEG)


def _tcbaac_prior(args=None):
    from ..tcbaac import CLASS_SEG, PRIOR_CLASSES, TiledCBAACCodec
    return TiledCBAACCodec(getattr(args, "order", 0) if args is not None else 0,
                           getattr(args, "segment_symbols", CLASS_SEG) if args is not None else CLASS_SEG, prior=True,
                           nclass=PRIOR_CLASSES)


# TCBAAC: CBAAC in independent segments on the GPU (vcf_amd/tcbaac.py, a new container);
# TCBAACP: the same with every segment's models seeded by a prior row of the frame: 8 rows, one per run of
# segments (about one subband row each), 4096-symbol segments (container version 3)
ENTROPY_CODECS = {"TIFF": TIFFCodec, "CBAAC": _cbaac, "CBAHC": _cbahc, "TCBAAC": _tcbaac, "TCBAACP": _tcbaac_prior}


def register_entropy_codec(name, cls):
    ENTROPY_CODECS[name] = cls


def make_entropy(args):
    """The entropy codec named by -c (no_filter.py:14-21)."""
    ec_name = getattr(args, "entropy_image_codec", "TIFF")
    if ec_name not in ENTROPY_CODECS:
        raise NotImplementedError(f"entropy codec {ec_name!r} (have: {sorted(ENTROPY_CODECS)})")
    maker = ENTROPY_CODECS[ec_name]
    return maker(args) if maker in (_cbaac, _cbahc, _tcbaac, _tcbaac_prior) else maker()


def make_quantizer(args):
    """None for -a deadzone (fused into the transform kernels), else the LloydMax plug-in."""
    quant = getattr(args, "quantizer", "deadzone")
    if quant == "deadzone":
        return None
    if quant == "LloydMax":
        return LloydMaxQuantizer(int(getattr(args, "QSS", 32)), int(getattr(args, "min_val", 0)),
                                 int(getattr(args, "max_val", 255)))
    raise NotImplementedError(f"quantizer {quant!r}: deadzone and LloydMax are on the HIP path")


class _Zipped:
    """A read TIFF whose strips the GPU inflates (decode_fns): the file bytes and
    its strip table (codec/tiff.py tiff_strips)."""

    def __init__(self, data: bytes, info):
        self.data, self.info = data, info

    def host(self) -> np.ndarray:
        from .tiff import imread_bytes
        return imread_bytes(self.data)


def _flags(args) -> int:
    return D.flags_from(bool(getattr(args, "disable_subbands", False)),
                        bool(getattr(args, "perceptual_quantization", False)))


class CoDec(EICCoDec):
    """2D-DCT.CoDec (2D-DCT.py:50-579) over the YCoCg / deadzone / no_filter /
    <entropy codec> chain."""

    def __init__(self, args):
        super().__init__(args)
        self.block_size = int(getattr(args, "block_size_DCT", 8))
        ct = getattr(args, "color_transform", "YCoCg")
        if ct not in ("YCoCg", "YCrCb"):
            raise NotImplementedError(f"color transform {ct!r}: YCoCg (and YCrCb, which 2D-DCT.py runs as "
                                      "YCoCg) are on the HIP path")
        self.lm = make_quantizer(args)
        filt = getattr(args, "filter", "no_filter")
        if not self.encoding and filt != "no_filter":
            raise NotImplementedError(f"filter {filt!r}: only no_filter is on the HIP path")
        if not D.block_size_supported(self.block_size):
            raise NotImplementedError(f"block size {self.block_size}: the HIP path covers 1 <= B <= 4096")
        self.entropy = make_entropy(args)
        self.file_extension = self.entropy.file_extension
        self.QSS = int(getattr(args, "QSS", 32))
        self.offset = 128 if self.lm is None else 0    # 2D-DCT.py:106-109
        self.flags = _flags(args)
        self.original_shape = None
        self.Lambda = None
        if self.encoding and getattr(args, "Lambda", None) is not None and self.lm is not None:
            raise NotImplementedError("-L with -a LloydMax: the search's quantizer calls are not on the HIP path")
        if self.encoding and getattr(args, "Lambda", None) is not None:
            # 2D-DCT.py:99-105
            if not getattr(args, "perceptual_quantization", False):
                self.Lambda = float(args.Lambda)
                logging.info("optimizing the block size")
                self.optimize_block_size()
                logging.info(f"optimal block_size={self.block_size}")
            else:
                logging.warning("sorry, perceptual quantization is only available for block_size=8")

    def bye(self):
        st = getattr(self, "_staged", None)
        if st is not None:
            st[1].close()
            self._staged = None
        super().bye()

    # entropy stage (TIFF.py / CBAAC.py surface)
    def compress(self, img):
        return self.entropy.compress(img)

    def decompress(self, codestream):
        return self.entropy.decompress(codestream)

    # 2D-DCT.py:187-266 semantics, used by callers that pad/crop themselves
    def pad_and_center_to_multiple_of_block_size(self, img):
        if img.ndim != 3:
            raise ValueError("Input image must be a 3D array (height, width, channels).")
        self.original_shape = img.shape
        H, W = img.shape[:2]
        Hp, Wp = D.padded_shape(H, W, self.block_size)
        t, l = (Hp - H) // 2, (Wp - W) // 2
        return np.pad(img, ((t, Hp - H - t), (l, Wp - W - l), (0, 0)), mode="constant")

    def remove_padding(self, padded_img):
        if padded_img.ndim != 3:
            raise ValueError("Padded image must be a 3D array (height, width, channels).")
        if self.original_shape is None:
            raise ValueError("Original shape is not set. Pad the image first.")
        H, W = self.original_shape[:2]
        t = (padded_img.shape[0] - H) // 2
        l = (padded_img.shape[1] - W) // 2
        return padded_img[t:t + H, l:l + W, :]

    # ---- -L: RD-optimized block size (2D-DCT.py:533-579) ---------------------
    def optimize_block_size(self, img: np.ndarray | None = None):
        """J = rate + Lambda * RMSE for B in 2, 4, ..., 128; the first minimum wins.

        As in the reference: the frame is encode_read()'s default
        /tmp/original.png (entropy_image_coding.py:67) unless given; the
        search runs inside __init__ before the deadzone offset of 128 is set
        (:99-109), so its offset is YCoCg's [0, 0, 0] (YCoCg.py:28-29) -- no
        -128 on the pixels, no +128 on k; the candidates always use the
        subband layout (get_subbands/get_blocks are unconditional there);
        rate = bytes of self.compress(uint8(k)); the reconstruction comes from
        the int32 k (no uint8 wrap), dequantized, IDCT'd and colour-converted
        in int32 (vcf_dct_dz_decode_k32); RMSE compares it with the input
        (:537, :572; A7).
        A11: for frame sides that are not multiples of B the reference hands
        the unpadded frame to DCT2D (unpinned); here each candidate pads and
        crops exactly as encode_fn/decode_fn do."""
        if img is None:
            img = self.encode_read()
        self._check_frame(img)
        H, W = img.shape[:2]
        x64 = img.astype(np.float32).astype(np.float64)   # img - [0, 0, 0]
        J_min = 1000000
        self.J = {}
        for block_size in [2 ** i for i in range(1, 8)]:
            k = D.encode_k32(img, self.QSS, 0, block_size)
            cs = self.compress(k.astype(np.uint8))
            cs.seek(0)
            rate = len(cs.read())
            y = D.decode_k32(k, H, W, self.QSS, 0, block_size)
            rmse = float(np.sqrt(np.mean((x64 - y) ** 2)))
            J = rate + self.Lambda * rmse
            self.J[block_size] = J
            logging.debug(f"J={J} for block_size={block_size}")
            if J < J_min:
                J_min = J
                self.block_size = block_size
        return self.block_size

    # ---- the hot path -------------------------------------------------------
    def _check_frame(self, img):
        if img.ndim != 3:
            raise ValueError("Input image must be a 3D array (height, width, channels).")
        if img.dtype != np.uint8 or img.shape[2] != 3:
            raise NotImplementedError(f"{img.dtype} x{img.shape[2]} images: the HIP path takes u8 RGB")

    def _deadzone_only(self, what):
        if self.lm is not None:
            raise NotImplementedError(f"{what} with -a LloydMax (use encode_fn/decode_fn)")

    def encode_lm(self, img: np.ndarray) -> np.ndarray:
        """2D-DCT.py:276-361 with -a LloydMax: offset 0, the float32 coefficients
        (subbands, -p) on the GPU, LloydMax.quantize_fn (side files at
        /tmp/encoded, as quantize_decom's default), k = float32 indices -> uint8 (:361)."""
        self._check_frame(img)
        self.original_shape = img.shape
        H, W = img.shape[:2]
        Hp, Wp = D.padded_shape(H, W, self.block_size)
        src = DeviceBuffer.from_array(img)
        coef = D.raw_encode_device(src, 1, H, W, self.flags, block_size=self.block_size)
        src.free()
        k = self.lm.quantize_device(coef, np.float32, Hp * Wp, 3, np.uint8)
        coef.free()
        self.total_output_size += self.lm.codebook_bytes   # LloydMax.py:107-108
        self.lm.codebook_bytes = 0
        out = k.download(np.empty((Hp, Wp, 3), np.uint8))
        k.free()
        return out

    def decode_lm(self, k: np.ndarray, shape) -> np.ndarray:
        """2D-DCT.py:399-466 with -a LloydMax: uint8 k -> int16, centroids (from /tmp/encoded's
        side files, LloydMax.dequantize_fn) truncated into int16, then the GPU synthesis, offset 0."""
        H, W = int(shape[0]), int(shape[1])
        Hp, Wp = D.padded_shape(H, W, self.block_size)
        k = np.ascontiguousarray(k, dtype=np.uint8)
        if k.shape != (Hp, Wp, 3):
            raise ValueError(f"index frame {k.shape} does not match {(Hp, Wp, 3)} for {H}x{W}")
        dk = DeviceBuffer.from_array(k)
        y = self.lm.dequantize_device(dk, np.uint8, Hp * Wp, 3, np.int16)
        dk.free()
        rgb = D.raw_decode_device(y, 1, H, W, self.flags, block_size=self.block_size)
        y.free()
        out = rgb.download(np.empty((H, W, 3), np.uint8))
        rgb.free()
        return out

    def encode_indices(self, img: np.ndarray) -> np.ndarray:
        """2D-DCT.py:276-361 on the GPU: u8 RGB -> u8 indices (k + 128, wrapped)."""
        self._deadzone_only("encode_indices")
        self._check_frame(img)
        self.original_shape = img.shape
        return D.encode(img, self.QSS, self.flags, self.block_size)

    def decode_indices(self, k: np.ndarray, shape) -> np.ndarray:
        """2D-DCT.py:399-466 on the GPU: u8 indices -> u8 RGB (padding removed)."""
        self._deadzone_only("decode_indices")
        H, W = int(shape[0]), int(shape[1])
        return D.decode(np.ascontiguousarray(k, dtype=np.uint8), H, W, self.QSS, self.flags,
                        self.block_size)

    def encode_fn(self, in_fn, out_fn):
        img = self.encode_read_fn(in_fn)
        if self.lm is not None:
            cs = self.compress(self.encode_lm(img))
        elif hasattr(self.entropy, "compress_device"):
            cs = self._encode_compress_device(img)
        else:
            cs = self.compress(self.encode_indices(img))
        with open(f"{out_fn}_shape.bin", "wb") as f:
            f.write(struct.pack("iii", *self.original_shape))
        return self.encode_write_fn(cs, out_fn)

    def _encode_compress_device(self, img):
        """GPU-resident entropy stage: the indices stay in HBM between the
        encode kernel and the coder (TCBAAC); only the code-stream comes back."""
        from ..device import DeviceBuffer
        self._check_frame(img)
        self.original_shape = img.shape
        H, W = img.shape[:2]
        Hp, Wp = D.padded_shape(H, W, self.block_size)
        coder = self.entropy.coder
        with coder.lock:     # the coder's stream is shared with other threads' calls
            src = DeviceBuffer.from_array(img, coder.stream)
            k = DeviceBuffer(Hp * Wp * 3)
            D.encode_device(src, 1, H, W, self.QSS, self.flags, out=k, stream=coder.stream,
                            block_size=self.block_size)
            return self.entropy.compress_device(k, (Hp, Wp, 3))

    def encode(self, in_fn="/tmp/original.png", out_fn="/tmp/encoded"):
        # 2D-DCT.py:374-375: the reference's encode() ignores -o/-e
        return self.encode_fn(in_fn, out_fn)

    def decode_fn(self, in_fn, out_fn):
        codestream = self.decode_read_fn(in_fn)
        with open(f"{in_fn}_shape.bin", "rb") as f:
            self.original_shape = struct.unpack("iii", f.read(12))
        k = self.decompress(codestream)
        if self.lm is not None:
            y = self.decode_lm(k, self.original_shape)
        else:
            y = self.decode_indices(k, self.original_shape)
        return self.decode_write_fn(y, out_fn)

    def decode(self, in_fn="/tmp/encoded", out_fn="/tmp/decoded.png"):
        return self.decode_fn(in_fn, out_fn)

    # ---- batched frames (III runner): one launch per batch of equal shapes --
    def encode_fns(self, pairs, batch: int = 64, io_threads: int = 16):
        """encode_fn over (in_fn, out_fn) pairs; returns the bytes written per
        frame.  A three-stage pipeline: host threads
        decode the PNGs of the next two batches while the GPU encodes this
        one (one launch per group of equal shapes), and TIFF deflate + file
        writes of the previous batches run behind it on the same pool.  When
        every input is a PNG of one shape the natively decodable kind, the
        frames go through pinned double-buffered slots (staging.StagedEncoder):
        decoded straight into page-locked memory, async copies, no stacking."""
        pairs = list(pairs)
        if not pairs:
            return []
        if self.lm is not None:   # one histogram and design per frame: frame by frame
            return [self.encode_fn(i, o) for i, o in pairs]
        staged = self._encode_fns_staged(pairs, batch, io_threads)
        if staged is not None:
            return staged
        sizes = [0] * len(pairs)
        batches = [pairs[b0:b0 + batch] for b0 in range(0, len(pairs), batch)]

        def _read(p):
            img = self.encode_read_fn(p[0])
            self._check_frame(img)
            return img

        def _write(out_fn, img_shape, k):
            with open(f"{out_fn}_shape.bin", "wb") as f:
                f.write(struct.pack("iii", *img_shape))
            return self.encode_write_fn(self.compress(k), out_fn)

        with ThreadPoolExecutor(max_workers=io_threads) as pool:
            reads = {}
            for b in range(min(2, len(batches))):
                reads[b] = [pool.submit(_read, p) for p in batches[b]]
            writes = []
            for b, chunk in enumerate(batches):
                imgs = [f.result() for f in reads.pop(b)]
                if b + 2 < len(batches):
                    reads[b + 2] = [pool.submit(_read, p) for p in batches[b + 2]]
                groups = {}
                for i, img in enumerate(imgs):
                    groups.setdefault(img.shape, []).append(i)
                ks = [None] * len(chunk)
                for shape, idx in groups.items():
                    out = D.encode(np.stack([imgs[i] for i in idx]), self.QSS, self.flags, self.block_size)
                    for j, i in enumerate(idx):
                        ks[i] = out[j]
                b0 = b * batch
                for i in range(len(chunk)):
                    writes.append((b0 + i, pool.submit(_write, chunk[i][1], imgs[i].shape, ks[i])))
                self.original_shape = imgs[-1].shape
            for i, f in writes:
                sizes[i] = f.result()
        return sizes

    def _encode_fns_staged(self, pairs, batch, io_threads):
        from .. import staging
        probes = [staging.png_probe(p[0]) if p[0].lower().endswith(".png") else None for p in pairs]
        if any(pr is None or not pr[2] for pr in probes) or len({pr[:2] for pr in probes}) != 1:
            return None
        H, W = probes[0][:2]
        batch = max(1, min(batch, len(pairs)))
        Hp, Wp = D.padded_shape(H, W, self.block_size)
        qss, flags, bsz = self.QSS, self.flags, self.block_size

        def launch(din, n, dout, stream):
            D.encode_device(din, n, H, W, qss, flags, out=dout, stream=stream, block_size=bsz)

        key = (batch, H, W, Hp, Wp, qss, flags, bsz)
        cached = getattr(self, "_staged", None)
        if cached is None or cached[0] != key:
            if cached is not None:
                cached[1].close()
            # pinning is costly (~0.1 s per GB): the slots live as long as the codec
            self._staged = (key, staging.StagedEncoder(batch, H, W, (Hp, Wp, 3), launch))
        enc = self._staged[1]
        sizes = [0] * len(pairs)
        batches = [pairs[b0:b0 + batch] for b0 in range(0, len(pairs), batch)]
        in_bytes = [0] * len(pairs)

        def _read(b, i):
            in_bytes[b * batch + i] = staging.decode_png_into(batches[b][i][0], enc.slot(b)["hin"].array[i])

        def _write(out_fn, k):
            with open(f"{out_fn}_shape.bin", "wb") as f:
                f.write(struct.pack("iii", H, W, 3))
            return self.encode_write_fn(self.compress(k), out_fn)

        # -c TIFF (the default): a batch's strips are deflated on the GPU from the
        # indices in HBM (vcf_amd/zlib_gpu.py, byte-exact with zlib), so only the
        # files come back; a single frame (encode_fn) keeps the host thread pool
        gpu_tiff = isinstance(self.entropy, TIFFCodec) and TIFFCodec.gpu_batches
        if gpu_tiff:
            from .. import zlib_gpu
            # rows over 64 KB (1-row strips past 21845 px) are beyond the GPU deflate's
            # strips: those frames keep the host writer
            gpu_tiff = zlib_gpu.covers((Hp, Wp, 3), 1)

        def _write_file(out_fn, blob):
            with open(f"{out_fn}_shape.bin", "wb") as f:
                f.write(struct.pack("iii", H, W, 3))
            return self.encode_write_fn(io.BytesIO(blob), out_fn)

        try:
            with ThreadPoolExecutor(max_workers=io_threads) as pool:
                reads = {0: [pool.submit(_read, 0, i) for i in range(len(batches[0]))]}
                writes = {}
                for b, chunk in enumerate(batches):
                    for f in reads.pop(b):
                        f.result()
                    # the other slot's pinned input is free (batch b-1 was copied in
                    # run(b-1)): decode the next batch's PNGs into it meanwhile
                    if b + 1 < len(batches):
                        reads[b + 1] = [pool.submit(_read, b + 1, i) for i in range(len(batches[b + 1]))]
                    # this slot's pinned output is still read by batch b-2's deflates
                    for i, f in writes.pop(b - 2, []):
                        sizes[i] = f.result()
                    if gpu_tiff:
                        from .. import zlib_gpu
                        dout, st = enc.run_device(b, len(chunk))
                        files = zlib_gpu.tiff_frames_device(dout, len(chunk), (Hp, Wp, 3), np.uint8, stream=st)
                        writes[b] = [(b * batch + i, pool.submit(_write_file, chunk[i][1], files[i]))
                                     for i in range(len(chunk))]
                        continue
                    ks = enc.run(b, len(chunk))
                    writes[b] = [(b * batch + i, pool.submit(_write, chunk[i][1], ks[i])) for i in range(len(chunk))]
                for lst in writes.values():
                    for i, f in lst:
                        sizes[i] = f.result()
        except BaseException:
            self._staged = None
            enc.close()
            raise
        self.total_input_size += sum(in_bytes)
        self.original_shape = (H, W, 3)
        return sizes

    def decode_fns(self, pairs, batch: int = 64, io_threads: int = 16):
        """decode_fn over (in_fn, out_fn) pairs, pipelined like encode_fns: the
        next two batches' TIFFs are inflated on host threads while the GPU
        decodes this one, and the PNG writes of earlier batches run behind."""
        pairs = list(pairs)
        if not pairs:
            return []
        if self.lm is not None:
            return [self.decode_fn(i, o) for i, o in pairs]
        sizes = [0] * len(pairs)
        batches = [pairs[b0:b0 + batch] for b0 in range(0, len(pairs), batch)]
        # -c TIFF (the default): a batch's strips are inflated on the GPU straight into
        # the index frames the decode kernel reads (vcf_amd/zlib_gpu.py StripInflater,
        # zlib.decompress's semantics); the host threads only read the files
        gpu_tiff = isinstance(self.entropy, TIFFCodec) and TIFFCodec.gpu_batches and self.block_size == 8

        def _read(p):
            cs = self.decode_read_fn(p[0])
            with open(f"{p[0]}_shape.bin", "rb") as f:
                shp = struct.unpack("iii", f.read(12))
            if gpu_tiff:
                from .tiff import tiff_strips
                info = tiff_strips(cs)
                Hp, Wp = D.padded_shape(shp[0], shp[1], self.block_size)
                if info is not None and tuple(info[0]) == (Hp, Wp, 3) and info[1] == np.uint8:
                    return _Zipped(cs, info), shp
            return self.decompress(cs), shp

        with ThreadPoolExecutor(max_workers=io_threads) as pool:
            reads = {b: [pool.submit(_read, p) for p in batches[b]] for b in range(min(2, len(batches)))}
            writes = []
            for b, chunk in enumerate(batches):
                got = [f.result() for f in reads.pop(b)]
                if b + 2 < len(batches):
                    reads[b + 2] = [pool.submit(_read, p) for p in batches[b + 2]]
                groups = {}
                for i, (k, shp) in enumerate(got):
                    groups.setdefault(tuple(shp), []).append(i)
                ys = [None] * len(chunk)
                for shp, idx in groups.items():
                    if all(isinstance(got[i][0], _Zipped) for i in idx):
                        out = self._decode_zipped([got[i][0] for i in idx], shp)
                    else:
                        ks = [got[i][0] if not isinstance(got[i][0], _Zipped) else got[i][0].host()
                              for i in idx]
                        out = D.decode(np.stack(ks), shp[0], shp[1], self.QSS, self.flags, self.block_size)
                    for j, i in enumerate(idx):
                        ys[i] = out[j]
                self.original_shape = got[-1][1]
                b0 = b * batch
                for i in range(len(chunk)):
                    writes.append((b0 + i, pool.submit(self.decode_write_fn, ys[i], chunk[i][1])))
            for i, f in writes:
                sizes[i] = f.result()
        return sizes

    def _decode_zipped(self, zs, shp):
        """n TIFFs of one shape -> n decoded frames: every strip inflated on the GPU
        into the index frames, the DCT + deadzone decode there, one download."""
        from ..device import Stream
        from .. import zlib_gpu
        H, W = shp[0], shp[1]
        Hp, Wp = D.padded_shape(H, W, self.block_size)
        fb, n = Hp * Wp * 3, len(zs)
        comp = np.frombuffer(b"".join(z.data for z in zs), np.uint8)
        base = np.concatenate([[0], np.cumsum([len(z.data) for z in zs])[:-1]]).astype(np.int64)
        comp_off = np.concatenate([b + np.asarray(z.info[2], np.int64) for b, z in zip(base, zs)])
        comp_len = np.concatenate([np.asarray(z.info[3], np.int32) for z in zs])
        sb = zs[0].info[4]
        ns = len(zs[0].info[2])
        if any(len(z.info[2]) != ns or z.info[4] != sb for z in zs):
            raise ValueError("TIFFs of one shape with different strip layouts")
        out_off = (np.arange(n, dtype=np.int64)[:, None] * fb + np.arange(ns, dtype=np.int64)[None, :] * sb).ravel()
        out_len = np.minimum(sb, fb - np.arange(ns, dtype=np.int64) * sb)
        out_len = np.tile(out_len, n).astype(np.int32)
        bufs = getattr(self, "_zdec", None)
        if bufs is None or bufs[0].nbytes < n * fb or bufs[1].nbytes < n * H * W * 3:
            bufs = self._zdec = (DeviceBuffer(n * fb), DeviceBuffer(n * H * W * 3), Stream())
        dk, drgb, st = bufs
        zlib_gpu.inflater().inflate_into(comp, comp_off, comp_len, dk, out_off, out_len, st)
        D.decode_device(dk, n, H, W, self.QSS, self.flags, out=drgb, stream=st, block_size=self.block_size)
        res = np.empty((n, H, W, 3), np.uint8)
        drgb.download(res, st)
        st.synchronize()
        return res

    # ---- quantizer surface (deadzone.py:95-124) -----------------------------
    def quantize_decom(self, decom):
        return self.quantize(decom)

    def dequantize_decom(self, decom_k):
        return self.dequantize(decom_k)

    def quantize(self, img, fn="/tmp/encoded"):
        if self.lm is not None:
            return self.lm.quantize(img, fn)
        from .. import quant
        return quant.deadzone_quantize(img, self.QSS)

    def dequantize(self, k, fn="/tmp/encoded"):
        if self.lm is not None:
            return self.lm.dequantize(k, fn)
        from .. import quant
        return quant.deadzone_dequantize(k, self.QSS)
