#!/usr/bin/env python3
"""Drop-in for `python 2D-DWT.py [-g] {encode,decode} [-l 5] [-w db5] ...`
(src/2D-DWT.py): YCoCg + dyadic 2D-DWT (mode 'per') + deadzone + TIFF
subbands, the hot span on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.dwt2d import CoDec  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402

if __name__ == "__main__":
    main(P.dwt_parser(entropy=P.entropy_of(sys.argv[1:])), CoDec)
