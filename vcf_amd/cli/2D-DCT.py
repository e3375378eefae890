#!/usr/bin/env python3
"""Drop-in for `python 2D-DCT.py [-g] {encode,decode} ...` (src/2D-DCT.py):
YCoCg + B x B DCT + deadzone (or -a LloydMax) + TIFF, the hot span on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.dct2d import CoDec  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402

if __name__ == "__main__":
    main(P.dct_parser(quantizer=P.quantizer_of(sys.argv[1:]), entropy=P.entropy_of(sys.argv[1:])), CoDec)
