"""AddressSanitizer + UndefinedBehaviorSanitizer build of the CPU oracle, driven through its
extraction (all 16 semantics variants), grid, SearchForInitialization, SearchByProjection, GetFeaturesInArea and
stereo entry points by tests/c/oracle_sanitize.c.  Host code only: GPU sanitizers are not available."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_ubsan(tmp_path):
    exe = tmp_path / "oracle_sanitize"
    src = [os.path.join(ROOT, "tests", "c", "oracle_sanitize.c"), os.path.join(ROOT, "oracle", "orb_oracle.c"),
           os.path.join(ROOT, "oracle", "oo_bow.c")]
    subprocess.check_call(["gcc", "-O1", "-g", "-std=c11", "-ffp-contract=off", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", *src, "-o", str(exe), "-lm"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "semantics variants exercised: 16" in r.stdout
    assert "ERROR" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
