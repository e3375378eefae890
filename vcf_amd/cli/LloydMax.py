#!/usr/bin/env python3
"""Drop-in for `python LloydMax.py [-g] {encode,decode} ...` (src/LloydMax.py):
per-channel Lloyd-Max quantization of the image, the per-pixel work on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402
from vcf_amd.codec.pixel import LloydMaxCoDec  # noqa: E402

if __name__ == "__main__":
    main(P.lloydmax_parser(entropy=P.entropy_of(sys.argv[1:])), LloydMaxCoDec)
