"""Build the gfx950 HIP library in-tree: orbslam2_with_quadrics_amd/liborbgpu.so.

hipcc cross-compiles for gfx950 without a GPU.  -ffp-contract=off keeps every float/double rounding
step of the reference explicit (the fused multiply-adds the reference build performs are written as
fmaf/fma in the source).  The .so is git-ignored but travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "liborbgpu.so")
SOURCES = ["orb_extract.hip", "orb_match.hip", "orb_stereo.hip", "orb_frame.hip", "orb_bow.hip", "orb_pins.hip",
           "orbgpu_capi.cpp"]
HEADERS = ["orbgpu_internal.h", "orbgpu_launch.h", "orb_math_dev.h", "orb_pattern.inc",
           os.path.join("..", "..", "include", "orbgpu.h")]
ARCH = os.environ.get("ORBGPU_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-Wall", "-Wno-unused-result", "-Wno-comment"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build the HIP library)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    for f in SOURCES + HEADERS + [os.path.basename(__file__)]:
        p = os.path.join(CSRC, f) if f != os.path.basename(__file__) else os.path.abspath(__file__)
        if os.path.exists(p) and os.path.getmtime(p) > t:
            return True
    return False


def build(force: bool = False, verbose: bool = False, defines=(), out: str | None = None) -> str:
    """Build liborbgpu.so (or, with `out`/`defines`, a timing variant of it: every remaining -D switch selects a bit-exact alternative)."""
    target = out or LIB
    if not force and out is None and not _stale():
        return LIB
    objs = []
    cc = hipcc()
    tmp = os.path.join(HERE, "build", os.path.basename(target))
    os.makedirs(tmp, exist_ok=True)
    for src in SOURCES:
        obj = os.path.join(tmp, src + ".o")
        cmd = [cc, f"--offload-arch={ARCH}", *FLAGS, *[f"-D{d}" for d in defines], "-x", "hip", "-c",
               os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        objs.append(obj)
    out_tmp = target + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out_tmp, *objs]
    subprocess.check_call(cmd)
    os.replace(out_tmp, target)
    return target


# ---- experiment / diagnostic builds of the same library (orbslam2_with_quadrics_amd/variants/liborbgpu_<name>.so).
# Every compile-time switch left in csrc/ is listed here with the build that flips it; build() of __graft_entry__
# builds them all, and tests/test_gpu_variants.py runs each one on the GPU and checks its keypoints, descriptors and
# matches bit-exactly against the default build's.
VARIANT_DIR = os.path.join(HERE, "variants")
VARIANTS = {
    "fastprof": ["OG_FAST_PROFILE=1"],        # FAST per-phase clocks (tools/fast_profile.py)
    "octprof0": ["OG_OCT_PROFILE=1"],         # octree per-round clocks of level 0 (tools/octree_profile.py)
    "octbt0": ["OG_OCT_BESTTAB=0"],           # octree final key pass instead of the cell-best table
}
# the run-time switches (environment variables read by liborbgpu.so), checked the same way with the default build
ENV_VARIANTS = {
    "forkall": {"ORBGPU_FORK_MIN_PIXELS": "0"},    # every small batch forks level 0 onto its own stream
    "forknone": {"ORBGPU_FORK_MIN_PIXELS": "1000000000000"},
    "forkbatch": {"ORBGPU_FORK_MAX_B": "1024"},    # every batch forks (measured -1 % at config 3, r06)
    "debugsync": {"ORBGPU_DEBUG_SYNC": "1"},       # synchronise after every stage (diagnostics)
}


def variant_path(name: str) -> str:
    return os.path.join(VARIANT_DIR, f"liborbgpu_{name}.so")


def build_variants(names=None) -> list:
    os.makedirs(VARIANT_DIR, exist_ok=True)
    return [build(force=True, defines=VARIANTS[n], out=variant_path(n)) for n in (names or VARIANTS)]


# ---- C++ host layer (ORB_SLAM2::ORBextractor / Frame / ORBmatcher / ORBVocabulary over the C ABI) ----
ROOT = os.path.dirname(HERE)
HOST_SRC = os.path.join(HERE, "host")
HOST_SOURCES = ["ORBextractor.cc", "Frame.cc", "ORBmatcher.cc", "ORBVocabulary.cc"]
HOST_LIB = os.path.join(HERE, "liborbslam2_gpu.so")
HOST_DRIVER = os.path.join(ROOT, "tests", "cpp", "host_parity")
# -ffp-contract=off: the host layer's own float arithmetic (mOw = -Rcw^T tcw) follows OpenCV's baseline
# build, which has no FMA
HOST_FLAGS = ["-O2", "-std=c++14", "-fPIC", "-ffp-contract=off", "-Wall", "-Wextra", "-Wno-unused-parameter",
              "-I", os.path.join(ROOT, "include")]


def build_host(verbose: bool = False) -> str:
    """Build liborbslam2_gpu.so (links liborbgpu.so, found next to it through $ORIGIN) and the parity driver
    tests/cpp/host_parity.  g++ only: the host layer holds no device code."""
    cxx = shutil.which("g++") or "g++"
    cmd = [cxx, *HOST_FLAGS, "-shared", "-o", HOST_LIB + ".tmp",
           *[os.path.join(HOST_SRC, f) for f in HOST_SOURCES],
           "-L", HERE, "-l:liborbgpu.so", "-Wl,-rpath,$ORIGIN", "-pthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(HOST_LIB + ".tmp", HOST_LIB)
    cmd = [cxx, *HOST_FLAGS, "-o", HOST_DRIVER + ".tmp", os.path.join(ROOT, "tests", "cpp", "host_parity.cc"),
           "-L", HERE, "-l:liborbslam2_gpu.so", "-l:liborbgpu.so",
           "-Wl,-rpath,$ORIGIN/../../orbslam2_with_quadrics_amd", "-pthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(HOST_DRIVER + ".tmp", HOST_DRIVER)
    return HOST_LIB


BINDING_RUNNER = os.path.join(ROOT, "tests", "binding_run", "run_binding")
MATCHER_RUNNER = os.path.join(ROOT, "tests", "binding_run", "run_matchers")
REFERENCE_INCLUDE = "/root/reference/include"


def build_binding_runner(verbose: bool = False):
    """Build the drop-in binding runners (test infrastructure), linked with liborbgpu.so:
    * tests/binding_run/run_binding: integration/ORBextractor.cc compiled against the reference's UNCHANGED
      include/ORBextractor.h with the test cv shim (integration/cvshim + tests/binding_run/cvmini.cc)
      (tests/test_gpu_binding_run.py);
    * tests/binding_run/run_matchers: the same extractor binding plus integration/ORBmatcher_perframe.cc and
      integration/Frame_stereo.cc, compiled against integration/refdecl (the reference declarations they use,
      checked line by line against the reference headers) with the test-only member definitions of
      tests/binding_run/refstubs.cc (tests/test_gpu_binding_matchers.py).
    Both need the reference headers, so they are built here (CPU container) and travel to the GPU box with the tree;
    returns None where the headers are absent."""
    if not os.path.exists(os.path.join(REFERENCE_INCLUDE, "ORBextractor.h")):
        return None
    cxx = shutil.which("g++") or "g++"
    flags = ["-O2", "-std=c++11", "-ffp-contract=off", "-Wall", "-Wextra", "-Wno-unused-parameter"]
    inc = ["-I", os.path.join(ROOT, "integration", "cvshim"), "-I", REFERENCE_INCLUDE, "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "integration")]
    link = ["-L", HERE, "-l:liborbgpu.so", "-Wl,-rpath,$ORIGIN/../../orbslam2_with_quadrics_amd", "-pthread"]
    br = os.path.join(ROOT, "tests", "binding_run")
    jobs = [
        (BINDING_RUNNER, inc, [os.path.join(ROOT, "integration", "ORBextractor.cc"), os.path.join(br, "cvmini.cc"),
                               os.path.join(br, "run_binding.cc")]),
        # refdecl first: its Frame.h / MapPoint.h / KeyFrame.h / ORBmatcher.h stand for the reference's (which need
        # Eigen / g2o); ORBextractor.h still comes from the reference
        (MATCHER_RUNNER, ["-I", os.path.join(ROOT, "integration", "refdecl"), "-I", br] + inc,
         [os.path.join(ROOT, "integration", f) for f in ("ORBextractor.cc", "ORBmatcher_perframe.cc", "Frame_stereo.cc")]
         + [os.path.join(br, f) for f in ("cvmini.cc", "refstubs.cc", "run_matchers.cc")]),
    ]
    for out, incs, srcs in jobs:
        cmd = [cxx, *flags, *incs, *srcs, *link, "-o", out + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(out + ".tmp", out)
    return BINDING_RUNNER


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_host(verbose=True))
