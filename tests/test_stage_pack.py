"""The add's range check and copy (foundationdb_amd/csrc/stage_pack.h, used by
TxnStage::add) against a plain restatement on random ranges -- point ranges,
short ranges, equal / reversed / prefix keys, lengths 0..100.  Host code: g++,
no GPU.  (The GPU tests check the same records end to end through the
verdicts.)"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_stage_pack_fuzz(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "stage_pack_fuzz")
    subprocess.run([gxx, "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "native", "stage_pack_fuzz.cpp")],
                   check=True)
    out = subprocess.run([exe, "40000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")
