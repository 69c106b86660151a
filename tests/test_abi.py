"""The drop-in boundary: librecsys_hip.so exists (built by __graft_entry__.build()), loads on
CPU, and exports every entry point include/recsys_hip.h declares; the ctypes table matches the
header one-to-one. No compute calls here (there is no GPU in the build container)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT, pkg

HEADER = os.path.join(ROOT, "include", "recsys_hip.h")
LIB = os.path.join(ROOT, "recommendation-system-maang-nvidia-_amd", "librecsys_hip.so")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rs_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_hot_path():
    fns = header_functions()
    for need in ("rs_embedding_gather_f32", "rs_sparse_adagrad_f32", "rs_gemm_f32", "rs_gemm_splitk_f32",
                 "rs_dcn_cross_vec_fwd_f32", "rs_dcn_cross_vec_bwd_f32", "rs_heads_fwd_f32",
                 "rs_heads_bwd_f32", "rs_ranking_losses_f32", "rs_inbatch_softmax_xent_fwd_f32",
                 "rs_inbatch_softmax_xent_bwd_f32", "rs_adagrad_dense_f32", "rs_topk_ip_f32"):
        assert need in fns


def test_ctypes_table_matches_header():
    native = pkg("_native")
    assert sorted(native.exported_symbols()) == header_functions()


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("librecsys_hip.so is not built; run __graft_entry__.build()")
    return pkg("_native").load()


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rs_[a-z0-9_]+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_abi_version_and_error_plumbing(lib):
    native = pkg("_native")
    assert lib.rs_abi_version() == native.ABI_VERSION
    # argument validation happens on the host before any HIP call: safe without a GPU
    with pytest.raises(native.NativeError, match="bad sizes"):
        native.call("rs_embedding_gather_f32", None, 0, 4, None, 0, None, None, None)
    assert "bad sizes" in lib.rs_last_error().decode()


def test_workspace_queries_are_host_only(lib):
    native = pkg("_native")
    assert native.query("rs_inbatch_softmax_workspace_bytes", 65536, 128) > 65536 * 128 * 4
    assert native.query("rs_gemm_splitk_workspace_bytes", 128, 256, 65536) > 0
    assert native.query("rs_topk_ip_workspace_bytes", 64, 1_000_000, 128, 100) > 0


def test_no_cpu_fallback_in_product_path():
    """The product ops refuse CPU tensors instead of silently computing elsewhere."""
    import torch
    F = pkg("functional")
    with pytest.raises(RuntimeError, match="ROCm device"):
        F.embedding_gather(torch.zeros((4, 4)), torch.zeros((2,), dtype=torch.int64))
    with pytest.raises(RuntimeError, match="ROCm device"):
        F.inbatch_softmax_fwd(torch.zeros((4, 32)), torch.zeros((4, 32)))
    src = open(os.path.join(ROOT, "recommendation-system-maang-nvidia-_amd", "functional.py")).read()
    assert "oracle" not in src


def test_reduction_queue_host_state():
    """rs_reduction_queue_* host bookkeeping (no GPU needed): the queue is caller-owned memory, an
    uninitialised or too small one is refused, nothing is queued without a reducing call, a flush of
    an empty queue is a no-op, and two queues are independent (the library keeps no queue state)."""
    import ctypes
    native = pkg("_native")
    n = native.query("rs_reduction_queue_bytes")
    assert 64 < n < 8192
    bufs = [(ctypes.c_uint64 * ((n + 7) // 8))() for _ in range(2)]
    q0, q1 = (ctypes.c_void_p(ctypes.addressof(b)) for b in bufs)
    assert native.query("rs_reduction_queue_pending", q0) == -1          # not initialised yet
    with pytest.raises(native.NativeError, match="not an initialised"):
        native.call("rs_reduction_queue_flush", q0, None)
    with pytest.raises(native.NativeError, match="need"):
        native.call("rs_reduction_queue_init", q0, n - 8)
    native.call("rs_reduction_queue_init", q0, ctypes.sizeof(bufs[0]))
    native.call("rs_reduction_queue_init", q1, ctypes.sizeof(bufs[1]))
    assert native.query("rs_reduction_queue_pending", q0) == 0
    assert native.query("rs_reduction_queue_pending", q1) == 0
    native.call("rs_reduction_queue_flush", q0, None)       # empty queue: no launch
    assert native.query("rs_reduction_queue_pending", q0) == 0
    assert not hasattr(native.load(), "rs_reductions_defer")   # the process-wide queue is gone


# every RS_* timing / A-B switch the kernels' host code has read (round 4's list plus the rest)
FORMER_ENV_SWITCHES = ("RS_MLP_ROWS", "RS_PGEMM_BM", "RS_GEMM_NO_SKINNY", "RS_GEMM_NO_WS", "RS_SPLITK_WANT",
                       "RS_XGEMM_VAR", "RS_IB_SPLIT_TARGET", "RS_SORT_LDS", "RS_SKINNY_WIDE_MASK", "RS_SKINNY_BLOCKS",
                       "RS_SKINNY_EPI_GENERIC", "RS_TOPK_RANGE_RATIO", "RS_TOPK_TWO_PHASE", "RS_TOPK_NT_LOADS",
                       "RS_TOPK_THR_W4", "RS_TOPK_EXP_TH_INF")


def test_release_library_reads_no_environment_switch():
    """Kernel selection is a function of the call's arguments (stateless): every
    getenv in csrc/ goes through common.hpp's exp_env, which is a getenv only in -DRS_EXPERIMENTS
    builds. So the sources call getenv nowhere else, and no switch name is left in the release .so."""
    csrc = os.path.join(ROOT, "recommendation-system-maang-nvidia-_amd", "csrc")
    for name in sorted(os.listdir(csrc)):
        if name.endswith(".hip"):
            src = open(os.path.join(csrc, name)).read()
            assert not re.search(r"(?<![a-z_])getenv\s*\(", src), name
    common = open(os.path.join(csrc, "common.hpp")).read()
    assert re.search(r"#ifdef RS_EXPERIMENTS.*getenv\(name\).*#else.*return nullptr", common, re.S)
    blob = open(LIB, "rb").read()
    left = [n for n in FORMER_ENV_SWITCHES if n.encode() in blob]
    assert not left, left


def test_python_layer_reads_no_kernel_selection_environment():
    """The Python host layer picks its paths from arguments, ModelConfig and module constants that
    only tests patch: os.environ is read only for the launcher's variables (distributed.py: RANK,
    WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, the backend override; trainer.py the same) and for the
    library's path (_native.py)."""
    pkg = os.path.join(ROOT, "recommendation-system-maang-nvidia-_amd")
    allowed = {"distributed.py": {"RANK", "WORLD_SIZE", "LOCAL_RANK", "RS_DIST_BACKEND", "MASTER_ADDR"},
               "trainer.py": {"WORLD_SIZE", "LOCAL_RANK"}, "_native.py": {"RECSYS_HIP_LIB"},
               "api.py": {"RS_MODEL_DIR"}}   # (the served model directory, app/main.py:113)
    for name in sorted(os.listdir(pkg)):
        if not name.endswith(".py"):
            continue
        src = open(os.path.join(pkg, name)).read()
        names = set(re.findall(r"os\.environ(?:\.get|\.setdefault)?\s*[\(\[]\s*\"([A-Z_]+)\"", src))
        assert names <= allowed.get(name, set()), (name, names - allowed.get(name, set()))
        assert "getenv" not in src, name
