"""A/B timing of run-time switches (environment variables read by liborbgpu.so) on the default library, GPU box.

Each named setting runs bench.py once (alternating settings for `--rounds` rounds) and prints frames/s, ms per step
and the parity field, so a switch is judged by the headline clock on the same box.

python tools/env_ab.py --set base: --set forkall:ORBGPU_FORK_MAX_B=1024 [--rounds 2] [-- extra bench args]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        extra = argv[argv.index("--") + 1:]
        argv = argv[:argv.index("--")]
    sets, rounds = [], 2
    i = 0
    while i < len(argv):
        if argv[i] == "--set":
            name, _, kv = argv[i + 1].partition(":")
            env = dict(x.split("=", 1) for x in kv.split(",") if x)
            sets.append((name, env))
            i += 2
        elif argv[i] == "--rounds":
            rounds = int(argv[i + 1])
            i += 2
        else:
            raise SystemExit(f"unknown argument {argv[i]}")
    for r in range(rounds):
        for name, env in sets:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", *extra]
            out = subprocess.run(cmd, env=dict(os.environ, **env), capture_output=True, text=True, timeout=600)
            try:
                js = json.loads(out.stdout.strip().splitlines()[-1])
                p = js.get("parity") or {}
                print(name, r, json.dumps(dict(value=js["value"], ms_per_step=js["ms_per_step"],
                                               parity=f"{p.get('frames')}/{p.get('mismatches')}")), flush=True)
            except Exception:
                print(name, r, "error", out.stderr[-600:], flush=True)


if __name__ == "__main__":
    main()
