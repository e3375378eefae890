#!/usr/bin/env python3
"""Drop-in for `python deadzone.py [-g] {encode,decode} ...` (src/deadzone.py): the image
quantized directly (int16, deadzone, uint8) on the GPU, then the entropy codec."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402
from vcf_amd.codec.pixel import DeadzoneCoDec  # noqa: E402

if __name__ == "__main__":
    main(P.deadzone_parser(entropy=P.entropy_of(sys.argv[1:])), DeadzoneCoDec)
