"""Host-side logic of the drop-in layer that needs no GPU: the config.json schema split, the
Keras-3 / Keras-2 EarlyStopping / ModelCheckpoint rules of the trainer, and the packed-batch tagging of the
hipGraph input copy."""
import json
import os

import numpy as np
import pytest

from conftest import oracle, pkg

HERE = os.path.dirname(os.path.abspath(__file__))


def test_config_json_keeps_the_reference_schema(tmp_path):
    """config.json must load through the reference's ModelConfig(**json.load(f))
    (src/models.py:98-102, app/model_service.py:40): exactly the src/config.py fields; the
    build-only fields round-trip through config_ext.json."""
    cfgm = pkg("config")
    ref_defaults = json.load(open(os.path.join(HERE, "golden", "config_defaults.json")))  # reference-run
    assert set(cfgm.REFERENCE_FIELDS) == set(ref_defaults)
    cfg = cfgm.ModelConfig(embedding_dim=32, cross_layers=1, contraction_precision=0, ctr_loss_mode="keras3",
                           clipnorm=0.5)
    cfgm.save_config(cfg, str(tmp_path))
    cj = json.load(open(tmp_path / "config.json"))
    assert set(cj) == set(ref_defaults)
    assert cj["embedding_dim"] == 32
    back = cfgm.load_config(str(tmp_path))
    assert back == cfg
    os.remove(tmp_path / "config_ext.json")              # a directory the reference wrote
    plain = cfgm.load_config(str(tmp_path))
    assert plain.embedding_dim == 32 and plain.contraction_precision == 6
    assert cfgm.load_config(str(tmp_path / "missing")) == cfgm.ModelConfig()


def _run_es(monitors, patience=3, mode="keras3"):
    tr = pkg("trainer")
    es = tr.EarlyStopping(patience=patience, mode=mode)
    log = []
    for epoch, m in enumerate(monitors):
        improved, stop = es.on_epoch_end(epoch, m, lambda e=epoch: {"epoch": e})
        log.append((improved, stop))
        if stop:
            break
    return es, log


@pytest.mark.parametrize("mode", ["keras3", "keras2"])
def test_early_stopping_rules(mode):
    # improvements checkpoint; a run that ends without triggering keeps its last weights under
    # Keras 2 and gets the best weights back under Keras 3 (on_train_end restore)
    es, log = _run_es([5.0, 4.0, 4.5, 3.0, 3.5], mode=mode)
    assert [i for i, _ in log] == [True, True, False, True, False]
    assert not any(s for _, s in log) and es.stopped_epoch == 0
    assert es.best_state == {"epoch": 3} and es.best == 3.0
    assert es.restore_at_end(False) == (mode == "keras3")
    assert es.restore_at_end(True)
    # no monitor value: nothing changes (Keras returns before counting the epoch)
    es, log = _run_es([None, None, None, None], patience=1, mode=mode)
    assert log == [(False, False)] * 4 and es.wait == 0 and not es.restore_at_end(False)
    # a NaN (never improving) monitor: Keras 3 records the first epoch's weights and restores them
    # at train end; Keras 2 has no best weights to restore
    es, log = _run_es([float("nan")] * 3, patience=5, mode=mode)
    assert log == [(False, False)] * 3 and es.wait == 3
    if mode == "keras3":
        assert es.best_state == {"epoch": 0} and es.best_epoch == 0 and es.restore_at_end(False)
    else:
        assert es.best_state is None and not es.restore_at_end(True)
    es, log = _run_es([float("nan"), 2.0, 3.0], patience=5, mode=mode)
    assert [i for i, _ in log] == [False, True, False] and es.best_state == {"epoch": 1}
    # patience 3: the third epoch without improvement stops and the best state is to be restored
    es, log = _run_es([5.0, 4.0, 4.1, 4.2, 4.3, 1.0])
    assert log[-1] == (False, True) and len(log) == 5 and es.stopped_epoch == 4
    assert es.best_state == {"epoch": 1}
    # an equal value is not an improvement (min_delta 0, mode 'min')
    es, log = _run_es([2.0, 2.0], patience=1)
    assert log == [(True, False), (False, True)]


def test_packed_batch_tagging():
    import torch
    graphs = pkg("graphs")
    feats = {"user_id": torch.arange(10), "movie_id": torch.arange(10) * 2}
    labels = {"rating": torch.ones(10), "y_implicit": torch.zeros(10)}
    pb = graphs.pack_batch((feats, labels))
    assert isinstance(pb, graphs.PackedBatch)
    assert graphs._packed_storage(pb) is not None
    assert torch.equal(pb[0]["movie_id"], feats["movie_id"]) and torch.equal(pb[1]["rating"], labels["rating"])
    # fields that merely share one big storage are NOT a packed batch (the static copy and the
    # replay memcpy would be the size of the whole storage)
    big = torch.zeros(4, 1000, dtype=torch.int64)
    sliced = ({"user_id": big[0, :10], "movie_id": big[1, :10]}, {})
    assert graphs._packed_storage(sliced) is None
    assert graphs._packed_storage(graphs.PackedBatch(sliced)) is None
    # copies between packed batches of different field shapes take the per-field path
    st = graphs._clone_batch(pb)
    other = graphs.pack_batch(({"user_id": torch.arange(10) + 5, "movie_id": torch.arange(10)}, labels))
    graphs._copy_into(st, other)
    assert torch.equal(st[0]["user_id"], torch.arange(10) + 5)
    assert not graphs._same_fields(st, graphs.pack_batch(({"user_id": torch.arange(12), "movie_id": torch.arange(8)},
                                                          labels)))


def test_bench_refuses_mislabelled_world():
    """bench.py --gpus N must measure N ranks: under a launcher whose WORLD_SIZE differs it exits
    non-zero before touching any GPU (without a launcher it starts the N ranks itself)."""
    import subprocess
    import sys
    root = os.path.dirname(HERE)
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=1" in r.stderr


def test_faiss_flat_index_file_layout(tmp_path):
    """faiss.idx as faiss.write_index lays out an IndexFlatIP / IndexFlatL2 (src/trainer.py:243,
    app/recommendation_service.py:47); parity unpinned (faiss is not importable): byte layout +
    round trip."""
    import struct
    fio = pkg("faiss_io")
    rng = np.random.default_rng(0)
    xb = rng.standard_normal((37, 16)).astype(np.float32)
    xb /= np.linalg.norm(xb, axis=1, keepdims=True)
    p = tmp_path / "faiss.idx"
    fio.write_index_flat(p, xb, "ip")
    raw = p.read_bytes()
    assert raw[:4] == b"IxFI"
    assert struct.unpack_from("<iqqqBiQ", raw, 4) == (16, 37, 1 << 20, 1 << 20, 1, 0, 37 * 16)
    assert len(raw) == 45 + 4 * 37 * 16
    metric, back = fio.read_index_flat(p)
    assert metric == "ip" and np.array_equal(back, xb)
    fio.write_index_flat(p, xb[:3], "l2")
    assert p.read_bytes()[:4] == b"IxF2" and fio.read_index_flat(p)[0] == "l2"
    p.write_bytes(b"IxHe" + raw[4:])
    with pytest.raises(ValueError, match="not a flat"):
        fio.read_index_flat(p)


def test_shuffle_buffer_order_matches_process_and_window():
    """make_ds's ds.shuffle(50000) (src/trainer.py:115-116) as the native shuffle-buffer order:
    bitwise the oracle's restatement of the process, a permutation, inside the window, fresh per
    epoch, deterministic in (seed, epoch). Host-only entry point (no GPU work)."""
    data, O = pkg("data"), oracle()
    for n, buf, seed, epoch in [(1, 1, 0, 0), (37, 5, 3, 1), (1000, 64, 7, 2), (500, 10_000, 1, 0),
                                (4096, 4096, 2, 5)]:
        got = data.shuffle_buffer_order(n, buf, seed, epoch).numpy()
        np.testing.assert_array_equal(got, O.shuffle_buffer_order(n, buf, seed, epoch))
        np.testing.assert_array_equal(np.sort(got), np.arange(n))
        assert (got < np.arange(n) + buf).all()
    np.testing.assert_array_equal(data.shuffle_buffer_order(100, 1).numpy(), np.arange(100))
    big = data.shuffle_buffer_order(200_000, 50_000, 0, 0).numpy()
    np.testing.assert_array_equal(np.sort(big), np.arange(200_000))
    assert (big < np.arange(200_000) + 50_000).all() and (big - np.arange(200_000)).max() > 40_000
    assert not np.array_equal(big, data.shuffle_buffer_order(200_000, 50_000, 0, 1).numpy())
    np.testing.assert_array_equal(big, data.shuffle_buffer_order(200_000, 50_000, 0, 0).numpy())
    assert data.shuffle_buffer_order(0, 50_000).numel() == 0
    with pytest.raises(pkg("_native").NativeError):
        data.shuffle_buffer_order(10, 0)


def test_reduction_queue_attachment_is_weak_and_replaceable():
    """a parameter holds only a weak reference to its optimizer's deferred-
    reduction queue; attaching another queue (a new optimizer) or none flushes and closes the old
    one, so an abandoned queue left open by an aborted step is never fed again; a dropped
    optimizer's queue disappears with it (host bookkeeping only, no GPU)."""
    import gc

    import torch
    F = pkg("functional")
    params = [torch.nn.Parameter(torch.zeros(3)) for _ in range(2)]
    q1 = F.ReductionQueue()
    F.attach_reduction_queue(params, q1)
    assert all(F._queue_of(p) is q1 for p in params)
    q1.open()                                # zero_grad() of a step that never reaches step()
    assert q1.active
    q2 = F.ReductionQueue()
    F.attach_reduction_queue(params, q2)      # a new deferring optimizer takes the parameters over
    assert not q1.active and all(F._queue_of(p) is q2 for p in params)
    q2.open()
    F.attach_reduction_queue(params, None)    # a non-deferring optimizer: nothing queues any more
    assert not q2.active and all(F._queue_of(p) is None for p in params)
    q3 = F.ReductionQueue()
    F.attach_reduction_queue(params, q3)
    del q3
    gc.collect()
    assert all(F._queue_of(p) is None for p in params)   # the owner is gone: no queue
    opt = pkg("optim").Adagrad(params, [], 0.1)            # CPU: never deferring, detaches
    assert opt._rq is None and all(F._queue_of(p) is None for p in params)
