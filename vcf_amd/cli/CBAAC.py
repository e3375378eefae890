#!/usr/bin/env python3
"""Drop-in for `python CBAAC.py [-g] {encode,decode} [--order N] ...` (src/CBAAC.py):
context-based adaptive arithmetic coding of the image (native coder, orders 0..8)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402
from vcf_amd.codec.pixel import CBAACImageCoDec  # noqa: E402

if __name__ == "__main__":
    main(P.cbaac_parser(), CBAACImageCoDec)
