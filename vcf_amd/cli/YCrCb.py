#!/usr/bin/env python3
"""Drop-in for `python YCrCb.py [-g] {encode,decode} ...` (src/YCrCb.py):
RGB -> YCrCb -> quantizer (-a deadzone or LloydMax), the per-pixel work on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402
from vcf_amd.codec.pixel import YCrCbCoDec  # noqa: E402

if __name__ == "__main__":
    main(P.ycrcb_parser(quantizer=P.quantizer_of(sys.argv[1:]), entropy=P.entropy_of(sys.argv[1:])), YCrCbCoDec)
