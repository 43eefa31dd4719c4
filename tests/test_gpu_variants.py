"""Every compile-time switch left in csrc/ is built (orbslam2_with_quadrics_amd/build_ext.py VARIANTS, prebuilt by
__graft_entry__.build()) and checked here on the GPU: the variant library's keypoints, descriptors and
SearchForInitialization matches on a 1080p, a KITTI-shaped and a VGA batch must equal the default build's bit for bit
(tests/variant_probe.py, one subprocess per library so each process loads exactly one liborbgpu).  The environment
switches (build_ext.ENV_VARIANTS) are checked the same way with the default library."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from orbslam2_with_quadrics_amd import build_ext  # noqa: E402

PROBE = os.path.join(ROOT, "tests", "variant_probe.py")


def _probe(lib, extra_env=None):
    env = dict(os.environ)
    env.pop("ORBGPU_LIB", None)
    for v in build_ext.ENV_VARIANTS.values():
        for k in v:
            env.pop(k, None)
    if lib:
        env["ORBGPU_LIB"] = lib
    env.update(extra_env or {})
    out = subprocess.run([sys.executable, PROBE], env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_digest():
    return _probe(None)


@pytest.mark.parametrize("name", sorted(build_ext.VARIANTS))
def test_variant_build_is_bit_exact(default_digest, name):
    lib = build_ext.variant_path(name)
    assert os.path.exists(lib), f"{lib} is not built (__graft_entry__.build() builds every variant)"
    got = _probe(lib)
    assert got == default_digest, (name, build_ext.VARIANTS[name])
    assert default_digest["hd"]["nmatches"] > 100


@pytest.mark.parametrize("name", sorted(build_ext.ENV_VARIANTS))
def test_runtime_switch_is_bit_exact(default_digest, name):
    """The run-time switches liborbgpu.so reads from the environment (block order, fork threshold, debug sync)."""
    got = _probe(None, build_ext.ENV_VARIANTS[name])
    assert got == default_digest, (name, build_ext.ENV_VARIANTS[name])
