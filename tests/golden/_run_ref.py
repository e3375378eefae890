"""Runs ONE reference encode_fn/decode_fn in-process under python3.9.

Invoked by make_golden.py as
    PYTHONPATH=tests/golden/shims:/root/reference/src python3.9 _run_ref.py \
        <module> <encode|decode> <in_fn> <out_fn> [reference CLI flags...]
The reference module is imported unmodified; its import-time argparse reads
sys.argv exactly as its CLI would (2D-DCT.py:47, deadzone.py:35, ...).
With VCF_GOLDEN_HIDE_IMAGECODECS=1 the optional imagecodecs package is hidden
so tifffile takes its stdlib-zlib path (level 6, tifffile.py:14971-14975),
as it does in an environment built from the reference's requirements.txt.
"""
import importlib
import os
import sys

if os.environ.get("VCF_GOLDEN_HIDE_IMAGECODECS") == "1":
    sys.modules["imagecodecs"] = None
import warnings

warnings.filterwarnings("ignore")

if os.environ.get("VCF_GOLDEN_LOG") == "1":
    # the reference's debug log (main.py:7-10) on stdout, message text only,
    # e.g. optimize_block_size's "J=... for block_size=..." (2D-DCT.py:576)
    import logging
    logging.basicConfig(format="LOG %(message)s", level=logging.DEBUG, stream=sys.stdout)

module, sub, in_fn, out_fn = sys.argv[1:5]
flags = sys.argv[5:]
sys.argv = [module + ".py", sub] + flags
mod = importlib.import_module(module)
import parser as ref_parser  # the reference's src/parser.py

args = ref_parser.parser.parse_known_args()[0]
codec = mod.CoDec(args)
fn = codec.encode_fn if sub == "encode" else codec.decode_fn
n = fn(in_fn, out_fn)
print(f"RESULT_BYTES {n}")
print(f"RESULT_BLOCK_SIZE {getattr(codec, 'block_size', None)}")
