"""Persistent autotuner table (ops/tune.TuneStore): round trip, identity invalidation, rank-0 broadcast."""
import json
import os

import torch.multiprocessing as mp

from pytorchvideo_accelerate_amd.ops.tune import TuneStore

IDENT = {"so": "abc", "device": "AMD Instinct MI355X", "hip": "7.0", "dtype": "bf16"}


def _tables():
    return {"conv": {}, "eval": {}, "wgrad": {}}


def test_round_trip_and_no_rewrite(tmp_path, monkeypatch):
    monkeypatch.setenv("PVA_TUNE_CACHE", str(tmp_path))
    t = _tables()
    st = TuneStore(t, IDENT)
    assert st.load() == 0
    t["conv"][("f", 8, 2, True, 100, 64, 576)] = 2048 | 16
    t["wgrad"][("w", 100, 64, 64, 8, 56, 56, 64, 576, 8, 2, False, 1, 3, 3, 1, 1, 1)] = 16 | 1024
    assert st.save() and not st.save()          # unchanged table: no rewrite
    t2 = _tables()
    st2 = TuneStore(t2, IDENT)
    assert st2.load() == 2 and t2 == t
    assert st2.path == st.path and os.path.dirname(st.path) == str(tmp_path)


def test_stale_identity_or_knob_invalidates(tmp_path, monkeypatch):
    monkeypatch.setenv("PVA_TUNE_CACHE", str(tmp_path))
    t = _tables()
    st = TuneStore(t, IDENT)
    t["conv"][("d", 1)] = 17
    st.save()
    assert TuneStore(_tables(), dict(IDENT, so="rebuilt")).load() == 0         # other .so build: other file
    monkeypatch.setenv("PVA_ARMS", "conv_direct=0")
    assert TuneStore(_tables(), IDENT).load() == 0                              # kernel-selection arm changed
    monkeypatch.delenv("PVA_ARMS")
    # a file whose recorded identity does not match (hash collision, hand edit) is ignored
    doc = json.load(open(st.path))
    doc["ident"]["so"] = "other"
    json.dump(doc, open(st.path, "w"))
    assert TuneStore(_tables(), IDENT).load() == 0
    monkeypatch.setenv("PVA_TUNE_CACHE", "0")
    assert not TuneStore(_tables(), IDENT).save(force=True)


def _rank(rank, world, port, root, out):
    import torch.distributed as dist
    from pytorchvideo_accelerate_amd.parallel.dist import DistState
    # rank 1 has no table of its own (another node's cache directory): it must receive rank 0's
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      PVA_TUNE_CACHE=root if rank == 0 else os.path.join(root, "rank1"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st = DistState(rank=rank, world_size=world, local_rank=rank, backend="gloo")
    t = _tables()
    ts = TuneStore(t, IDENT)
    doc = st.broadcast_object(ts.read() if rank == 0 else None)
    n = ts.restore(doc)
    out[rank] = (n, sorted(map(str, t["conv"].items())))
    dist.destroy_process_group()


def test_rank0_table_broadcast(tmp_path, monkeypatch):
    import socket
    monkeypatch.setenv("PVA_TUNE_CACHE", str(tmp_path))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    t = _tables()
    st = TuneStore(t, IDENT, root=str(tmp_path))
    t["conv"][("f", 1, 2)] = 16
    st.save()
    out = mp.Manager().dict()
    mp.spawn(_rank, args=(2, port, str(tmp_path), out), nprocs=2)
    assert out[0] == out[1] == (1, [str((("f", 1, 2), 16))])
