"""faiss.idx for the flat inner-product / L2 index the reference writes (src/trainer.py:236-245:
faiss.normalize_L2(embs); IndexFlatIP(d); add; faiss.write_index) and its serving path reads
(app/recommendation_service.py:47, faiss.read_index) — without faiss, which is not importable here.

On-disk layout of faiss's write_index for an IndexFlat (faiss/impl/index_write.cpp; the same bytes
from faiss 1.5 to 1.8: the older WRITEVECTOR of a float vector and the newer WRITEXBVECTOR of the
code bytes both store the float count as a size_t, then the floats), little-endian:
    fourcc        4 B   "IxFI" (METRIC_INNER_PRODUCT) / "IxF2" (METRIC_L2)
    d             int32
    ntotal        int64
    dummy, dummy  int64, int64 (both 1 << 20)
    is_trained    uint8 (1)
    metric_type   int32 (0 = inner product, 1 = L2)
    n             uint64 = ntotal * d
    xb            n float32, row-major [ntotal][d]
Parity unpinned: faiss is absent, so the format is checked by round trips and by this byte layout
only (tests/test_host_cpu.py), not against a file faiss itself wrote.
"""
from __future__ import annotations

import struct
from typing import Tuple

import numpy as np

_FOURCC = {"ip": b"IxFI", "l2": b"IxF2"}
_METRIC = {"ip": 0, "l2": 1}


def write_index_flat(path, xb: np.ndarray, metric: str = "ip") -> None:
    """faiss.write_index(IndexFlatIP / IndexFlatL2 holding xb, path)."""
    if metric not in _FOURCC:
        raise ValueError(f"metric must be 'ip' or 'l2', got {metric!r}")
    xb = np.ascontiguousarray(np.asarray(xb, dtype=np.float32))
    if xb.ndim != 2:
        raise ValueError("xb must be [ntotal, d]")
    n, d = xb.shape
    with open(path, "wb") as f:
        f.write(_FOURCC[metric])
        f.write(struct.pack("<iqqq", d, n, 1 << 20, 1 << 20))
        f.write(struct.pack("<Bi", 1, _METRIC[metric]))
        f.write(struct.pack("<Q", n * d))
        f.write(xb.astype("<f4", copy=False).tobytes())


def read_index_flat(path) -> Tuple[str, np.ndarray]:
    """faiss.read_index of a flat IP / L2 index -> (metric 'ip' | 'l2', xb [ntotal, d] float32)."""
    with open(path, "rb") as f:
        buf = f.read()
    h = buf[:4]
    metric = {v: k for k, v in _FOURCC.items()}.get(h)
    if metric is None:
        raise ValueError(f"{path}: not a flat IP/L2 faiss index (fourcc {h!r})")
    d, n, _, _ = struct.unpack_from("<iqqq", buf, 4)
    trained, mt = struct.unpack_from("<Bi", buf, 32)
    if mt != _METRIC[metric] or not trained:
        raise ValueError(f"{path}: metric {mt} / is_trained {trained} inconsistent with {h!r}")
    off = 37
    if mt > 1:                                   # metric_arg (not used by IP / L2)
        off += 4
    (cnt,) = struct.unpack_from("<Q", buf, off)
    off += 8
    if cnt != n * d or len(buf) != off + 4 * cnt:
        raise ValueError(f"{path}: {cnt} floats for ntotal={n}, d={d}, file size {len(buf)}")
    xb = np.frombuffer(buf, dtype="<f4", count=cnt, offset=off).reshape(n, d).astype(np.float32)
    return metric, xb
