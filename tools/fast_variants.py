"""Timing experiments for the FAST cells kernel (test infrastructure).  Builds variants of liborbgpu.so
that stop the kernel after a given stage (OG_EXP_FAST_STOP=1: ROI load, 2: quick test + survivor list,
3: exact score + NMS count; 0 = full kernel) into orbslam2_with_quadrics_amd/variants/, and -- with
--run on the GPU box -- times each with bench.py's per-stage HIP events.  Variant results are wrong by
construction; only the FAST stage time is read.

python tools/fast_variants.py --build            # here (hipcc cross-compiles)
python tools/fast_variants.py --run              # on the GPU box
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "orbslam2_with_quadrics_amd", "variants")
VARIANTS = {"full": [], "stop_roi": ["OG_EXP_FAST_STOP=1"], "stop_quick": ["OG_EXP_FAST_STOP=2"],
            "stop_count": ["OG_EXP_FAST_STOP=3"], "nostage": ["OG_EXP_FAST_NOSTAGE=1"]}
EXTRA = json.loads(os.environ.get("FAST_VARIANTS_EXTRA", "{}"))
VARIANTS.update(EXTRA)


def build():
    from orbslam2_with_quadrics_amd import build_ext

    os.makedirs(VDIR, exist_ok=True)
    for name, defs in VARIANTS.items():
        print(build_ext.build(force=True, defines=defs, out=os.path.join(VDIR, f"liborbgpu_{name}.so")))


def run():
    res = {}
    for name in VARIANTS:
        env = dict(os.environ, ORBGPU_LIB=os.path.join(VDIR, f"liborbgpu_{name}.so"))
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "2", "--streams", "1",
                              "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
        try:
            js = json.loads(out.stdout.strip().splitlines()[-1])
            res[name] = js["stages_ms_per_launch"]
        except Exception:
            res[name] = {"error": out.stderr[-800:]}
        print(name, res[name], flush=True)
    return res


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    if "--run" in sys.argv:
        r = run()
        if "--json" in sys.argv:
            json.dump(r, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
