"""vcf_amd -- MI355X-native implementation of VCF's per-frame hot path.

YCoCg colour transform -> 8x8 block DCT -> deadzone quantizer (fused HIP
kernels for gfx950, bit-exact to the reference's numpy/scipy path), entropy
coding (TIFF/deflate host stage) and the reference's encode()/decode() plugin
surface (vcf_amd.codec) and CLI (vcf_amd/cli).  See DESIGN.md.
"""
from ._lib import VCFError, VCFInvalidArgument, VCFUnsupported, lib  # noqa: F401

__version__ = "0.1.0"
