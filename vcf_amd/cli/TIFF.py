#!/usr/bin/env python3
"""Drop-in for `python TIFF.py [-g] {encode,decode} ...` (src/TIFF.py): the image itself
through the TIFF entropy codec (zlib strips, byte-exact with tifffile 2021.7.2)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402
from vcf_amd.codec.pixel import TIFFImageCoDec  # noqa: E402

if __name__ == "__main__":
    main(P.tiff_parser(), TIFFImageCoDec)
