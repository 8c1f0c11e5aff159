"""The DPP wave helpers of csrc/train_dev.h (wave_sum_u32, wave_max_u64,
wave_scan_incl_u32) against plain loops, lane by lane, on the GPU: every
training kernel's reductions and scans use them."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-bpe_amd", "lib", "dpp_check")


def test_dpp_wave_helpers():
    assert os.path.exists(BIN), "gpu-bpe_amd/lib/dpp_check missing: run __graft_entry__.build() (make -C gpu-bpe_amd)"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "dpp_check: ok" in r.stdout, r.stdout + r.stderr
