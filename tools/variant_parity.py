"""Parity of experiment builds (test infrastructure, GPU box): for every library in orbslam2_with_quadrics_amd/variants/
(or --names a,b), extract a few seeded frames and compare keypoints + descriptors bit for bit with the CPU oracle.

python tools/variant_parity.py [--names a,b]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "orbslam2_with_quadrics_amd", "variants")
CHILD = r'''
import sys, numpy as np
sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + "/oracle")
import torch
import oracle_py as O
from orbslam2_with_quadrics_amd import ORBextractor, synthetic
res = []
for (H, W, nf, seed) in ((1080, 1920, 2000, 21), (1080, 1920, 4000, 60), (480, 640, 1000, 22), (376, 1241, 2000, 5)):
    img = synthetic.frame(seed, H, W)
    k, d = ORBextractor(nf, 1.2, 8, 20, 7, device=0)(img)
    ko, do = O.OracleExtractor(nf)(img)
    res.append(dict(shape=f"{W}x{H}/{nf}", n=len(k), n_oracle=len(ko),
                    kps_equal=bool(len(k) == len(ko) and k.tobytes() == ko.tobytes()),
                    desc_equal=bool(d.shape == do.shape and np.array_equal(d, do))))
print("RESULT", json.dumps(res))
'''


def main():
    names = sorted(f[len("liborbgpu_"):-3] for f in os.listdir(VDIR) if f.startswith("liborbgpu_") and f.endswith(".so"))
    if "--names" in sys.argv:
        names = sys.argv[sys.argv.index("--names") + 1].split(",")
    for name in names:
        lib = os.path.join(ROOT, "orbslam2_with_quadrics_amd", "liborbgpu.so") if name == "default" else \
            os.path.join(VDIR, f"liborbgpu_{name}.so")
        env = dict(os.environ, ORBGPU_LIB=lib)
        out = subprocess.run([sys.executable, "-c", "import json\nROOT=%r\n" % ROOT + CHILD], env=env,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("RESULT ")]
        print(name, line[0][7:] if line else "ERROR " + out.stderr[-800:], flush=True)


if __name__ == "__main__":
    main()
