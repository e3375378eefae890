#!/usr/bin/env python3
"""Drop-in for `python III.py [-g] {encode,decode} [-T 2D-DCT] [-N 20] ...`
(src/III.py).  Multi-GPU: launch one process per GPU with
`python -m torch.distributed.run --nproc-per-node N vcf_amd/cli/III.py ...`;
frames are sharded in contiguous chunks."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from vcf_amd.codec import parser as P  # noqa: E402
from vcf_amd.codec.iii import CoDec  # noqa: E402
from vcf_amd.codec.main import main  # noqa: E402

if __name__ == "__main__":
    # the reference imports the -T codec module, whose options join the parser
    t = P.parse(P.iii_parser(), sys.argv[1:]).transform if len(sys.argv) > 1 else "2D-DCT"
    main(P.iii_parser(transform=t, entropy=P.entropy_of(sys.argv[1:])), CoDec)
