#!/usr/bin/env python3
"""Drop-in for `python YCoCg.py [-g] {encode,decode} ...` (src/YCoCg.py): RGB -> int16 YCoCg ->
quantizer (-a deadzone: one fused GPU kernel per direction; or LloydMax) -> uint16 -> entropy codec."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402
from vcf_amd.codec.pixel import YCoCgCoDec  # noqa: E402

if __name__ == "__main__":
    main(P.ycocg_parser(quantizer=P.quantizer_of(sys.argv[1:]), entropy=P.entropy_of(sys.argv[1:])), YCoCgCoDec)
