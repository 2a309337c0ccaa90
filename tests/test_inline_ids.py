"""The inline id of a digit STRING key (ksql_amd/csrc/khip_inline_id.hpp, the SWAR form the
kernels run) against a byte-by-byte restatement, compiled for the host with g++."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_inline_ids_swar_matches_bytewise(tmp_path):
    exe = str(tmp_path / "inline_ids_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "ksql_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "inline_ids_check.cpp"), "-o", exe], check=True)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 mismatches" in p.stdout
