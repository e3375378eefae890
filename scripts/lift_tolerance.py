"""Measure the opt-in lifting DWT's float64 coefficients against pywt's
(oracle restatement) on the lifting tests' frames and one 4K frame; prints
one JSON line (committed under profiles/)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import vcf_amd.dwt as DW
from oracle import lift_tolerance as LT
from vcf_amd.synthetic import synth_frame

rng = np.random.Generator(np.random.PCG64(7))
frames = {"synthetic_270x480": synth_frame(270, 480, 3),
          "noise_270x480": rng.integers(0, 256, (270, 480, 3), dtype=np.uint8),
          "noise_133x251": rng.integers(0, 256, (133, 251, 3), dtype=np.uint8),
          "white_270x480": np.full((270, 480, 3), 255, np.uint8),
          "synthetic_2160x3840": synth_frame(2160, 3840, 9)}
res = {name: LT.compare(DW.lift_coefficients(f, 5), f, 5) for name, f in frames.items()}
print(json.dumps({"what": "lifting bior4.4 l=5 float64 coefficients vs pywt 'per' (oracle), before quantization",
                  "frames": res}))
