"""Bounds-checked debug build (``python build.py --debug-bounds`` -> ``_C_dbg``, loaded with
``JLA_DEBUG_BOUNDS=1``): out-of-range indices that come from device state are clamped or skipped exactly as
in the release build, AND recorded in an error word the host reads (``ops.bounds_error`` /
``ops.check_bounds``). SURVEY.md section 5 (race detection / sanitizers: "debug build flag for
bounds-checked kernels").

The debug checks run in a child process (the release ``_C`` stays loaded in this one). The bad indices
used here are ones the kernels clamp or skip, so no out-of-bounds access is ever made.
"""
from __future__ import annotations

import glob
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, torch
from jax_llama_amd import ops
e = ops.ext()
res = {"debug": bool(e.DEBUG_BOUNDS), "so": e.__file__}
dev = "cuda"
ops.bounds_error(reset=True)
# clean run: nothing recorded
table = torch.randn(100, 256, device=dev).to(torch.bfloat16)
ids = torch.tensor([0, 5, 99], dtype=torch.int32, device=dev)
ops.embedding(ids, table)
torch.cuda.synchronize()
res["clean"] = ops.bounds_error(reset=True)
# token id past the vocabulary: clamped to the last row (as in release) and recorded
out = ops.embedding(torch.tensor([3, 100], dtype=torch.int32, device=dev), table)
res["clamped_row_ok"] = bool(torch.equal(out[1].cpu(), table[99].float().cpu()))
res["token"] = ops.bounds_error(reset=True)
# KV-cache write at a slot past the cache: skipped (cache untouched) and recorded
B, S, H, Hkv, Dh, T = 1, 2, 4, 2, 128, 8
qkv = torch.randn(B * S, (H + 2 * Hkv) * Dh, device=dev).to(torch.bfloat16)
rope = torch.randn(64, Dh // 2, 2, device=dev)
pos = torch.arange(S, dtype=torch.int32, device=dev)
kc = torch.zeros(B, Hkv, T, Dh, device=dev, dtype=torch.bfloat16)
vc = torch.zeros_like(kc)
ops.rope_kv_write(qkv, rope, pos, kc, vc, T - 1, S, H, Hkv, Dh)  # second row lands at slot T
torch.cuda.synchronize()
res["kv"] = ops.bounds_error(reset=True)
res["slot_T_minus_1_written"] = bool(kc[0, :, T - 1].abs().sum().item() > 0)
try:
    ops.embedding(torch.tensor([-1], dtype=torch.int32, device=dev), table)
    ops.check_bounds()
    res["raised"] = False
except ops.BoundsError as ex:
    res["raised"] = "vocabulary" in str(ex)
print("RESULT " + json.dumps(res))
"""


def _dbg_so():
    return glob.glob(os.path.join(ROOT, "jax_llama_amd", "_C_dbg*.so"))


def test_release_build_reports_no_debug():
    from jax_llama_amd import ops
    assert not ops.ext().DEBUG_BOUNDS
    assert ops.bounds_error() == 0
    ops.check_bounds()  # no-op


@pytest.mark.skipif(not _dbg_so(), reason="debug build absent (python build.py --debug-bounds)")
def test_debug_build_records_out_of_range_indices():
    env = dict(os.environ, JLA_DEBUG_BOUNDS="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["debug"] and "_C_dbg" in res["so"]
    assert res["clean"] == 0
    assert res["clamped_row_ok"]
    assert res["token"] == 1 << 0
    assert res["kv"] == 1 << 1
    assert res["slot_T_minus_1_written"]
    assert res["raised"]
