"""Shared test plumbing.

Markers: `gpu` = needs a ROCm GPU (MI355X) and the built librecsys_hip.so; everything else runs
on CPU. The parity tests compare the HIP path with the oracle (oracle/recsys_oracle.py, a numpy
restatement of the reference arithmetic) on the same seeded inputs.
"""
import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKG_NAME = "recommendation-system-maang-nvidia-_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")


def pkg(sub=None):
    name = PKG_NAME if sub is None else f"{PKG_NAME}.{sub}"
    return importlib.import_module(name)


def oracle():
    return importlib.import_module("oracle.recsys_oracle")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    pkg("_native").load()  # fail loudly if the extension is missing on a GPU box
    return torch.device("cuda")


def rel_err(a, b, floor=1.0):
    """max |a - b| / max(floor, max |b|): absolute error for O(1) values, relative to the
    tensor's scale for large ones (floor=0 makes it purely scale-relative)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        raise AssertionError(f"shape mismatch {a.shape} vs {b.shape}")
    if not a.size:
        return 0.0
    den = max(floor, float(np.max(np.abs(b))))
    if den == 0.0:
        den = 1.0
    return float(np.max(np.abs(a - b))) / den


def assert_close(a, b, tol=1e-4, what="", floor=1.0):
    e = rel_err(a, b, floor)
    assert e <= tol, f"{what}: max|a-b|/max({floor},|b|max) = {e:.3e} > {tol:.1e}"


# ---------------------------------------------------------------------------------------------
# ReLU gates of the GPU forward, for comparing against the oracle under the same activation
# pattern (oracle masks= instrument): an fp32 pre-activation within rounding of zero can take the
# other side of zero from the float64 one, and a hot id repeated ~1000 times in a batch multiplies
# that one unit's gradient contribution; under shared gates the comparison is at the fp32 bar.
# ---------------------------------------------------------------------------------------------
SCORE_SLOT = np.array([(u & 3) | ((u >> 1) & 4) | ((u << 1) & 8) for u in range(16)])


def score_tiles(buf):
    """Kept-score tiles -> [..., user, item] blocks of 32 x 32. A tile (1024 floats, inbatch.hip
    'Score-tile layout') holds S(user u, item i) at 512 (u / 16) + 16 i + ib_slot(u % 16), ib_slot
    swapping bits 2 and 3. buf: [..., 1024]."""
    b = np.asarray(buf).reshape(buf.shape[:-1] + (2, 32, 16))[..., SCORE_SLOT]   # [.., half, item, u%16]
    return np.swapaxes(b, -1, -2).reshape(buf.shape[:-1] + (32, 32))


def stack_gates(layers, rec, require_backward=True):
    """The ReLU gates (bool ndarray per ReLU layer) one Dense stack's node applied in the step run
    under functional.record_relu_gates() (its own forward's saved outputs, whatever kernels it ran),
    after checking them against that step's backward: every ReLU layer's pre-activation gradient is
    zero outside its gate, i.e. these are the gates the backward used."""
    key = layers[0].kernel.data_ptr()
    assert key in rec["fwd"], "the stack's node did not run under the recorder"
    gates = rec["fwd"][key]
    relu_idx = [k for k, layer in enumerate(layers) if layer.activation == "relu"]
    assert len(gates) == len(relu_idx)
    sup = rec["bwd"].get(key, {})
    if require_backward:
        assert sorted(sup) == relu_idx, (sorted(sup), relu_idx)
    for j, k in enumerate(relu_idx):
        if k in sup:
            assert not bool((sup[k] & ~gates[j]).any()), f"layer {k}: gradient outside the recorded gate"
    return [g.cpu().numpy() for g in gates]


def gpu_relu_masks(model, rec, require_backward=True):
    """{"user_tower", "item_tower", "deep": [bool ndarray per ReLU layer]}: the gates a
    MultiTaskModel step run under functional.record_relu_gates() applied (stack_gates)."""
    enc = model.encoder
    return {"user_tower": stack_gates(enc.user_tower.layers, rec, require_backward),
            "item_tower": stack_gates(enc.item_tower.layers, rec, require_backward),
            "deep": stack_gates(model.dcn.deep_nets, rec, require_backward)}


def mask_flips(O, P, ocfg, uid, iid, masks):
    """Units whose float64 pre-activation (the oracle forward under `masks`) lies on the other
    side of zero from the gate: {stack: [(count, max |pre| / scale over them)]}, scale = sum_k
    |x_k W_kj| + |b_j| (the size of the terms whose fp32 rounding decides the sign)."""
    c = O.forward(P, ocfg, uid, iid, masks)
    out = {}
    for key, acts, names, relu_last in (("user_tower", c["u_acts"], O.tower_names(ocfg, "user_tower"), False),
                                        ("item_tower", c["i_acts"], O.tower_names(ocfg, "item_tower"), False),
                                        ("deep", c["d_acts"], O.deep_names(ocfg), True)):
        res = []
        for j, (kn, bn) in enumerate(names):
            if not relu_last and j == len(names) - 1:
                continue
            W, b = P[kn], P[bn]
            pre = acts[j] @ W + b
            scale = np.abs(acts[j]) @ np.abs(W) + np.abs(b)
            flip = (pre > 0) != masks[key][j]
            ratio = float(np.max(np.abs(pre[flip]) / np.maximum(scale[flip], 1e-300))) if flip.any() else 0.0
            res.append((int(flip.sum()), ratio))
        out[key] = res
    return out


def assert_flips_are_rounding(flips, bound=1e-5):
    """Every gate that disagrees with the float64 sign sits within fp32 rounding of zero."""
    for key, layers in flips.items():
        for j, (n, ratio) in enumerate(layers):
            assert ratio <= bound, f"{key} layer {j}: {n} flipped units, |pre|/scale up to {ratio:.2e}"
