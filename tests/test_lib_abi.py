"""CPU tests: the C-ABI library builds/loads and exports every symbol include/orbgpu.h declares
(no compute calls -- there is no GPU here); the product path fails loudly without a device."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "orbgpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(orbgpu_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from orbslam2_with_quadrics_amd import _lib, build_ext

    build_ext.build()
    L = _lib.lib(load_torch_first=False)
    decl = declared_symbols()
    assert len(decl) >= 30
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(_lib.EXPORTS) == decl


def test_no_gpu_means_loud_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from orbslam2_with_quadrics_amd import ORBextractor

    with pytest.raises(RuntimeError):
        ORBextractor(1000, 1.2, 8, 20, 7)


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "orbslam2_with_quadrics_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(dp, f), errors="ignore").read()
                assert "oracle_py" not in src and "orb_oracle" not in src, f


def test_header_compiles_as_c(tmp_path):
    import subprocess

    c = tmp_path / "t.c"
    c.write_text('#include "orbgpu.h"\nint main(void){orbgpu_keypoint k; (void)k; return sizeof(orbgpu_keypoint)!=28;}\n')
    exe = tmp_path / "t"
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c), "-o",
                           str(exe)])
    subprocess.check_call([str(exe)])
