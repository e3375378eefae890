#!/usr/bin/env python3
"""Drop-in for `python CBAHC.py [-g] {encode,decode} [--order N] ...` (src/CBAHC.py):
context-based adaptive Huffman coding of the image (native coder)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402
from vcf_amd.codec.pixel import CBAHCImageCoDec  # noqa: E402

if __name__ == "__main__":
    main(P.cbahc_parser(), CBAHCImageCoDec)
