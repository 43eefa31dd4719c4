"""A/B timing of experiment builds of liborbgpu.so (test infrastructure, GPU box).

Runs bench.py once per library in orbslam2_with_quadrics_amd/variants/ (ORBGPU_LIB selects it) and prints the
frames/s and the per-stage HIP-event times of each, so a kernel change is judged by the same clock as the
headline number.  Build variants here first, e.g. with build_ext.build(defines=[...], out=...).

python tools/variant_bench.py [--streams S] [--names a,b,...] [--json out.json] [-- extra bench args]

A name may carry environment settings for its run: `lib@KEY=VAL:KEY2=VAL2` (e.g. `head@ORBGPU_FORK_MAX_B=1024`).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "orbslam2_with_quadrics_amd", "variants")


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        extra = argv[argv.index("--") + 1:]
        argv = argv[:argv.index("--")]
    streams = argv[argv.index("--streams") + 1] if "--streams" in argv else "2"
    names = sorted(f[len("liborbgpu_"):-3] for f in os.listdir(VDIR) if f.startswith("liborbgpu_") and f.endswith(".so"))
    if "--names" in argv:
        names = argv[argv.index("--names") + 1].split(",")
    res = {}
    for name in names:
        lib, _, sets = name.partition("@")
        env = dict(os.environ, ORBGPU_LIB=os.path.join(VDIR, f"liborbgpu_{lib}.so"))
        env.update(kv.split("=", 1) for kv in sets.split(":") if kv)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--warmup", "2", "--streams", streams,
               "--no-cpu-baseline", *extra]
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        try:
            js = json.loads(out.stdout.strip().splitlines()[-1])
            res[name] = dict(value=js["value"], ms_per_step=js["ms_per_step"], stages=js["stages_ms_per_launch"],
                             parity=js.get("parity"))
        except Exception:
            res[name] = {"error": out.stderr[-600:]}
        print(name, json.dumps(res[name]), flush=True)
    if "--json" in argv:
        json.dump(res, open(argv[argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
