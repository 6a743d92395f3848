"""The device walks DeviceShare's identical per-resource hint lists as one list (ks_numa.h): the exhaustive
check in tools/merge_collapse_check.c runs the oracle's merge both ways over the whole finite case space."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_identical_device_lists_merge_as_one(tmp_path):
    exe = tmp_path / "merge_collapse_check"
    subprocess.run(["gcc", "-O2", "-o", str(exe), os.path.join(ROOT, "tools", "merge_collapse_check.c"),
                    os.path.join(ROOT, "oracle", "koord_oracle.c"), os.path.join(ROOT, "oracle", "cpu_accumulator.c"),
                    "-I", os.path.join(ROOT, "include"), "-lm", "-lpthread"], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert out.strip().endswith("mismatches 0"), out
    assert int(out.split("cases")[1].split()[0]) > 400_000
