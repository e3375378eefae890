"""Runs ONE reference module as its own program, exactly as
`python <module>.py [flags] {encode,decode}` would, under python3.9:

    PYTHONPATH=tests/golden/shims:/root/reference/src python3.9 _run_ref_main.py \\
        <module> [reference CLI flags...]

runpy executes src/<module>.py with __name__ == "__main__", so module-level
`if __name__ == "__main__"` blocks run too (CBAAC.py:158-166 adds --order
there).  encode()/decode() use entropy_image_coding's hard-wired files
(/tmp/original.png -> /tmp/encoded<ext> -> /tmp/decoded.png, :19-22); the
caller stages the input and collects the outputs.
"""
import os
import runpy
import sys
import warnings

warnings.filterwarnings("ignore")
if os.environ.get("VCF_GOLDEN_HIDE_IMAGECODECS") == "1":
    sys.modules["imagecodecs"] = None

module = sys.argv[1]
path = os.path.join(os.getcwd(), module + ".py")
sys.argv = [path] + sys.argv[2:]
sys.path.insert(0, os.getcwd())
runpy.run_path(path, run_name="__main__")
