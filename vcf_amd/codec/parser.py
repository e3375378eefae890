"""Command-line surface of the reference, built explicitly.

The reference assembles its argparse parser from import side effects: every
module in the codec chain adds its options to the shared `parser.parser`
(src/parser.py:61-81) and then imports the next module named by an option
(2D-DCT.py -> YCoCg.py -> deadzone.py -> no_filter.py -> TIFF.py ->
entropy_image_coding.py).  Here the same options -- names, flags, defaults,
help -- are added by plain functions, so a Namespace from this parser has
exactly the attributes the reference's CoDec classes read (the Namespaces
printed in notebooks/III.ipynb cells 8 and 13).
"""
from __future__ import annotations

import argparse

# defaults (module constants of the reference)
ORIGINAL = "/tmp/original.png"          # entropy_image_coding.py:19
ENCODED = "/tmp/encoded"                # :20 (extension decided at run time)
DECODED = "/tmp/decoded.png"            # :22
DEFAULT_BLOCK_SIZE = 8                  # 2D-DCT.py:27
DEFAULT_CT = "YCoCg"                    # :28
DEFAULT_QUANTIZER = "deadzone"          # YCoCg.py:15
DEFAULT_QSS = 32                        # deadzone.py:23
DEFAULT_FILTER = "no_filter"            # deadzone.py:26
DEFAULT_EIC = "TIFF"                    # no_filter.py:11
DEFAULT_TRANSFORM = "2D-DCT"            # video_coding.py:33
N_FRAMES = 20                           # video_coding.py:31
DEFAULT_LEVELS = 5                      # 2D-DWT.py
DEFAULT_WAVELET = "db5"                 # 2D-DWT.py:23


def int_or_str(text):
    """src/parser.py:4-9."""
    try:
        return int(text)
    except ValueError:
        return text


def _encode(codec):
    return codec.encode()


def _decode(codec):
    return codec.decode()


class CustomArgumentParser(argparse.ArgumentParser):
    """src/parser.py:17-28: print the message and exit with the status."""

    def exit(self, status=0, message=None):
        if message:
            self._print_message(message, None)
        raise SystemExit(status)


def base_parser(description: str | None = None):
    """src/parser.py:63-81: -g and the encode/decode subcommands."""
    p = CustomArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter,
                             exit_on_error=False, description=description)
    p.add_argument("-g", "--debug", action="store_true", help="Output debug information")
    sub = p.add_subparsers(help="You must specify one of the following subcomands:",
                           dest="subparser_name")
    enc = sub.add_parser("encode", help="Compress data")
    dec = sub.add_parser("decode", help="Uncompress data")
    enc.set_defaults(func=_encode)
    dec.set_defaults(func=_decode)
    return p, enc, dec


def add_eic(enc, dec):
    """entropy_image_coding.py:25-30."""
    enc.add_argument("-o", "--original", type=int_or_str,
                     help=f"Input image (default: {ORIGINAL})", default=ORIGINAL)
    enc.add_argument("-e", "--encoded", type=int_or_str,
                     help=f"Output image (default: {ENCODED})", default=f"{ENCODED}")
    dec.add_argument("-e", "--encoded", type=int_or_str,
                     help=f"Input code-stream (default: {ENCODED})", default=f"{ENCODED}")
    dec.add_argument("-d", "--decoded", type=int_or_str,
                     help=f"Output image (default: {DECODED})", default=f"{DECODED}")


def add_filter(enc, dec, entropy: str = DEFAULT_EIC):
    """no_filter.py:14-21 (entropy codec choice lives in the filter module; the
    module -c names is imported there, and CBAHC.py adds --order on import)."""
    enc.add_argument("-c", "--entropy_image_codec",
                     help=f"Entropy Image Codec (default: {DEFAULT_EIC})", default=DEFAULT_EIC)
    dec.add_argument("-c", "--entropy_image_codec",
                     help=f"Entropy Image Codec (default: {DEFAULT_EIC})", default=DEFAULT_EIC)
    if entropy == "CBAHC":
        add_order_cbahc(enc, dec)


DEFAULT_ORDER = 0                       # CBAHC.py:13


def add_order_cbahc(enc, dec):
    """CBAHC.py:13-16 (at import time)."""
    for p in (enc, dec):
        p.add_argument("--order", type=int, help=f"Context model order (default: {DEFAULT_ORDER})",
                       default=DEFAULT_ORDER)


def add_order_cbaac(enc, dec):
    """CBAAC.py:158-164 (only when CBAAC.py itself is the program: as a -c
    module its CoDec reads getattr(args, 'order', 0), :76)."""
    for p in (enc, dec):
        p.add_argument("--order", type=int, default=0, help="Context order")


def entropy_of(argv) -> str:
    """Pre-parse -c/--entropy_image_codec, as the reference's import chain does (no_filter.py:20-21)."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("-c", "--entropy_image_codec", default=DEFAULT_EIC)
    return pre.parse_known_args(argv)[0].entropy_image_codec


def add_deadzone(enc, dec):
    """deadzone.py:32-35."""
    enc.add_argument("-q", "--QSS", type=int_or_str,
                     help=f"Quantization step size (default: {DEFAULT_QSS})", default=DEFAULT_QSS)
    dec.add_argument("-q", "--QSS", type=int_or_str,
                     help=f"Quantization step size (default: {DEFAULT_QSS})", default=DEFAULT_QSS)
    dec.add_argument("-f", "--filter", type=int_or_str,
                     help=f"Denoising filter (default: {DEFAULT_FILTER})", default=DEFAULT_FILTER)


def add_lloydmax(enc, dec):
    """LloydMax.py:27-35: -q as deadzone's, plus -m/--min_val and -n/--max_val (and -f on decode)."""
    add_deadzone(enc, dec)
    for p in (enc, dec):
        p.add_argument("-m", "--min_val", type=int_or_str, help="Default min_val (default: 0)", default=0)
        p.add_argument("-n", "--max_val", type=int_or_str, help="Default max_val (default: 255)", default=255)


def add_quantizer(enc, dec, quantizer: str = DEFAULT_QUANTIZER):
    """The options of the module -a names (YCoCg.py:21 imports it)."""
    if quantizer == "LloydMax":
        add_lloydmax(enc, dec)
    else:
        add_deadzone(enc, dec)


def quantizer_of(argv) -> str:
    """Pre-parse -a/--quantizer, as the reference's import chain does (YCoCg.py:20-21)."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("-a", "--quantizer", default=DEFAULT_QUANTIZER)
    return pre.parse_known_args(argv)[0].quantizer


def add_ycocg(enc, dec):
    """YCoCg.py:17-19."""
    enc.add_argument("-a", "--quantizer", help=f"Quantizer (default: {DEFAULT_QUANTIZER})",
                     default=DEFAULT_QUANTIZER)
    dec.add_argument("-a", "--quantizer", help=f"Quantizer (default: {DEFAULT_QUANTIZER})",
                     default=DEFAULT_QUANTIZER)


def add_dct(enc, dec):
    """2D-DCT.py:34-45."""
    for p, what in ((enc, "quantization"), (dec, "dequantization")):
        p.add_argument("-B", "--block_size_DCT", type=int_or_str,
                       help=f"Block size (default: {DEFAULT_BLOCK_SIZE})", default=DEFAULT_BLOCK_SIZE)
        p.add_argument("-t", "--color_transform", type=int_or_str,
                       help=f"Color transform (default: \"{DEFAULT_CT}\")", default=DEFAULT_CT)
        p.add_argument("-p", "--perceptual_quantization", action="store_true",
                       help=f"Use perceptual {what} (default: \"False\")", default=False)
        if p is enc:
            p.add_argument("-L", "--Lambda", type=int_or_str,
                           help="Relative weight between the rate and the distortion. If provided "
                                "(float), the block size is RD-optimized between {2**i; i=1,2,3,4,5,6,7}. "
                                "For example, if Lambda=1.0, then the rate and the distortion have the "
                                "same weight.")
        p.add_argument("-x", "--disable_subbands", action="store_true",
                       help="Disable the coefficients reordering in subbands (default: \"False\")",
                       default=False)


def add_dwt(enc, dec):
    """2D-DWT.py:25-31."""
    for p in (enc, dec):
        p.add_argument("-l", "--levels", type=int_or_str,
                       help=f"Number of decomposition levels (default: {DEFAULT_LEVELS})", default=DEFAULT_LEVELS)
        p.add_argument("-w", "--wavelet", type=int_or_str,
                       help=f"Wavelet name (default: \"{DEFAULT_WAVELET}\")", default=DEFAULT_WAVELET)
        p.add_argument("-t", "--color_transform", type=int_or_str,
                       help=f"Color transform (default: \"{DEFAULT_CT}\")", default=DEFAULT_CT)


def add_iii(enc, dec):
    """III.py:23-33."""
    for p, what in ((enc, "encode"), (dec, "decode")):
        p.add_argument("-T", "--transform", type=str,
                       help=f"2D-transform, default: {DEFAULT_TRANSFORM}", default=DEFAULT_TRANSFORM)
        p.add_argument("-N", "--number_of_frames", type=int_or_str,
                       help=f"Number of frames to {what} (default: {N_FRAMES})", default=f"{N_FRAMES}")


def dct_parser(description: str = "Exploiting spatial redundancy with the 2D Discrete Cosine "
                                  "Transform of constant block size.", quantizer: str = DEFAULT_QUANTIZER,
               entropy: str = DEFAULT_EIC):
    """The parser `python 2D-DCT.py ...` ends up with (the codec chain -a and -c name)."""
    p, enc, dec = base_parser(description)
    add_dct(enc, dec)
    add_ycocg(enc, dec)
    add_quantizer(enc, dec, quantizer)
    add_filter(enc, dec, entropy)
    add_eic(enc, dec)
    return p


def dwt_parser(description: str = "Exploiting spatial redundancy with the 2D dyadic Discrete Wavelet "
                                  "Transform.", entropy: str = DEFAULT_EIC):
    """`python 2D-DWT.py ...` (2D-DWT.py -> YCoCg.py -> deadzone.py -> no_filter.py -> TIFF.py)."""
    p, enc, dec = base_parser(description)
    add_dwt(enc, dec)
    add_ycocg(enc, dec)
    add_deadzone(enc, dec)
    add_filter(enc, dec, entropy)
    add_eic(enc, dec)
    return p


def iii_parser(description: str = "III coding: runs a 2D image codec for each image of a sequence.",
               transform: str = "2D-DCT", entropy: str = DEFAULT_EIC):
    """`python III.py ...` (III.py + the chain of the 2D codec it imports)."""
    p, enc, dec = base_parser(description)
    add_iii(enc, dec)
    if transform == "2D-DWT":
        add_dwt(enc, dec)
    else:
        add_dct(enc, dec)
    add_ycocg(enc, dec)
    add_deadzone(enc, dec)
    add_filter(enc, dec, entropy)
    add_eic(enc, dec)
    return p


def lloydmax_parser(description: str = "Image quantization using a LloydMax quantizer.",
                    entropy: str = DEFAULT_EIC):
    """`python LloydMax.py ...` (LloydMax.py -> no_filter.py -> TIFF.py)."""
    p, enc, dec = base_parser(description)
    add_lloydmax(enc, dec)
    add_filter(enc, dec, entropy)
    add_eic(enc, dec)
    return p


def ycrcb_parser(description: str = "Exploiting color (perceptual) redundancy with the YCrCb transform.",
                 quantizer: str = DEFAULT_QUANTIZER, entropy: str = DEFAULT_EIC):
    """`python YCrCb.py ...` (YCrCb.py -> <quantizer>.py -> no_filter.py -> TIFF.py)."""
    p, enc, dec = base_parser(description)
    add_ycocg(enc, dec)        # YCrCb.py:17-19 adds the same -a option
    add_quantizer(enc, dec, quantizer)
    add_filter(enc, dec, entropy)
    add_eic(enc, dec)
    return p


def ycocg_parser(description: str = "Exploiting color (perceptual) redundancy with the YCoCg transform.",
                 quantizer: str = DEFAULT_QUANTIZER, entropy: str = DEFAULT_EIC):
    """`python YCoCg.py ...` (YCoCg.py:15-21 -> <quantizer>.py -> no_filter.py -> TIFF.py)."""
    return ycrcb_parser(description, quantizer, entropy)


def deadzone_parser(description: str = "Image quantization using a deadzone scalar quantizer.",
                    entropy: str = DEFAULT_EIC):
    """`python deadzone.py ...` (deadzone.py:32-35 -> no_filter.py -> TIFF.py)."""
    p, enc, dec = base_parser(description)
    add_deadzone(enc, dec)
    add_filter(enc, dec, entropy)
    add_eic(enc, dec)
    return p


def tiff_parser(description: str = "Entropy Encoding of images using TIFF (Tag Image File Format). "):
    """`python TIFF.py ...` (TIFF.py -> entropy_image_coding.py)."""
    p, enc, dec = base_parser(description)
    add_eic(enc, dec)
    return p


def cbaac_parser(description: str = "Context-based adaptive arithmetic coding"):
    """`python CBAAC.py ...` (CBAAC.py -> entropy_image_coding.py, then --order, :158-164)."""
    p, enc, dec = base_parser(description)
    add_eic(enc, dec)
    add_order_cbaac(enc, dec)
    return p


def cbahc_parser(description: str = "\n# Huffman adaptativo\n"):
    """`python CBAHC.py ...` (CBAHC.py:13-16 --order, then entropy_image_coding.py)."""
    p, enc, dec = base_parser(description)
    add_order_cbahc(enc, dec)
    add_eic(enc, dec)
    return p


def parse(parser, argv=None):
    """parser.parse_known_args()[0] as main.py:9 does."""
    return parser.parse_known_args(argv)[0]


def add_ipp(enc, dec):
    """IPP_DCT.py:45-130 (the --st pre-parser and the temporal options)."""
    for p in (enc, dec):
        p.add_argument("--st", dest="space_transform", type=str, default="2D-DCT",
                       help="Spatial transform codec (default: 2D-DCT)")
    enc.add_argument("-i", "--input", type=str, default=IPP_INPUT, help=f"Input video (default: {IPP_INPUT})")
    enc.add_argument("-O", "--output", type=str, default=IPP_OUTPUT, help=f"Output prefix (default: {IPP_OUTPUT})")
    enc.add_argument("-N", "--number_of_frames", type=int, default=IPP_N_FRAMES,
                     help=f"Number of frames to encode (default: {IPP_N_FRAMES})")
    enc.add_argument("-G", "--gop_size", type=int, default=IPP_GOP, help=f"GOP size for IPP pattern (default: {IPP_GOP})")
    enc.add_argument("-M", "--block_size_ME", type=int, default=IPP_BLOCK_ME,
                     help=f"Motion estimation block size (default: {IPP_BLOCK_ME})")
    enc.add_argument("-S", "--search_range", type=int, default=IPP_SEARCH,
                     help=f"Search range in pixels (default: {IPP_SEARCH})")
    enc.add_argument("--fast", action="store_true", help="Use fast motion estimation (3-step search)")
    enc.add_argument("--threads", type=int, default=0, help="Number of threads (0=auto, default: 0)")
    enc.add_argument("-R", "--rdo_lambda", type=float, default=0.0,
                     help="RDO lambda for IPP block mode decision (default: 0.0)")
    dec.add_argument("-i", "--input", type=str, default=IPP_OUTPUT, help=f"Input prefix (default: {IPP_OUTPUT})")
    dec.add_argument("-O", "--output", type=str, default="./ipp_decoded", help="Output prefix (default: ./ipp_decoded)")
    dec.add_argument("-N", "--number_of_frames", type=int, default=IPP_N_FRAMES,
                     help=f"Number of frames (default: {IPP_N_FRAMES})")
    dec.add_argument("-G", "--gop_size", type=int, help="GOP size for IPP pattern")
    dec.add_argument("-M", "--block_size_ME", type=int, help="Motion estimation block size")
    dec.add_argument("-S", "--search_range", type=int, help="Search range in pixels")


IPP_INPUT = "http://www.hpca.ual.es/~vruiz/videos/mobile_352x288x30x420x300.mp4"   # IPP_DCT.py:36
IPP_OUTPUT = "./ipp_encoded"
IPP_N_FRAMES = 30
IPP_GOP = 10
IPP_BLOCK_ME = 16
IPP_SEARCH = 8


def ipp_parser(description: str = "IPP hybrid video coding using motion compensation and DCT.",
               space_transform: str = "2D-DCT", entropy: str = DEFAULT_EIC):
    """`python IPP_DCT.py ...` over the 2D-DCT chain (or, --st 2D-DWT, the 2D-DWT one)."""
    p, enc, dec = base_parser(description)
    if space_transform == "2D-DWT":
        add_dwt(enc, dec)
    else:
        add_dct(enc, dec)
    add_ycocg(enc, dec)
    add_deadzone(enc, dec)
    add_filter(enc, dec, entropy)
    add_eic(enc, dec)
    add_ipp(enc, dec)
    return p
