"""Runs ONE reference codec's encode()/decode() in-process under python3.9,
for the stand-alone codecs whose methods take no file names (YCrCb.py:33-72,
LloydMax.py:56-73: encode() reads encode_read()'s default /tmp/original.png
and writes encode_write()'s default /tmp/encoded, entropy_image_coding.py:67-82).

    PYTHONPATH=tests/golden/shims:/root/reference/src python3.9 _run_ref_codec.py \
        <module> <encode|decode> <in_fn> <out_fn> [reference CLI flags...]

The module is imported unmodified; only the instance's four default-path
wrappers are rebound to in_fn/out_fn (they are one-line calls of the *_fn
methods in the reference).  The quantizers' own side files keep the
reference's hard-wired prefix /tmp/encoded (LloydMax.py:116, :139).
"""
import importlib
import os
import sys
import warnings

warnings.filterwarnings("ignore")
if os.environ.get("VCF_GOLDEN_HIDE_IMAGECODECS") == "1":
    sys.modules["imagecodecs"] = None

module, sub, in_fn, out_fn = sys.argv[1:5]
flags = sys.argv[5:]
sys.argv = [module + ".py", sub] + flags
mod = importlib.import_module(module)
import parser as ref_parser  # the reference's src/parser.py

args = ref_parser.parser.parse_known_args()[0]
codec = mod.CoDec(args)
if sub == "encode":
    codec.encode_read = lambda fn=None: codec.encode_read_fn(in_fn)
    codec.encode_write = lambda cs, fn=None: codec.encode_write_fn(cs, out_fn)
    n = codec.encode()
else:
    codec.decode_read = lambda fn=None: codec.decode_read_fn(in_fn)
    codec.decode_write = lambda img, fn=None: codec.decode_write_fn(img, out_fn)
    n = codec.decode()
print(f"RESULT_BYTES {n}")
