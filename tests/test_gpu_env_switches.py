"""The release library ignores the RS_* switches its kernels' host code once read from the
environment (SURVEY §8b 'stateless'): the same product calls, run in a fresh process
with every former switch set to a non-default value, give bitwise the same outputs."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT
from test_abi import FORMER_ENV_SWITCHES

# a non-default value for each switch (what an A/B run of the experiment build would set)
SETTINGS = {"RS_MLP_ROWS": "32", "RS_PGEMM_BM": "256", "RS_GEMM_NO_SKINNY": "1", "RS_GEMM_NO_WS": "1",
            "RS_SPLITK_WANT": "64", "RS_XGEMM_VAR": "3", "RS_IB_SPLIT_TARGET": "256", "RS_SORT_LDS": "0",
            "RS_SKINNY_WIDE_MASK": "1", "RS_SKINNY_BLOCKS": "2", "RS_SKINNY_EPI_GENERIC": "1",
            "RS_TOPK_RANGE_RATIO": "8", "RS_TOPK_TWO_PHASE": "0", "RS_TOPK_NT_LOADS": "1", "RS_TOPK_THR_W4": "1",
            "RS_TOPK_EXP_TH_INF": "1"}


def _digest(extra_env):
    env = {k: v for k, v in os.environ.items() if k not in SETTINGS}
    env.update(extra_env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "env_switch_probe.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("DIGEST")]
    assert line, r.stdout[-2000:]
    return line[-1].split()[1]


@pytest.mark.gpu
def test_former_env_switches_change_nothing():
    import torch
    if torch.cuda.device_count() == 0:   # (counting devices does not initialise the GPU here)
        pytest.skip("no ROCm GPU visible")
    assert sorted(SETTINGS) == sorted(FORMER_ENV_SWITCHES)
    assert _digest({}) == _digest(SETTINGS)
