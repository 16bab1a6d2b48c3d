"""N > 1 path on CPU with gloo, world_size 2: weight broadcast from rank 0, image sharding,
token gather (the only collectives of the multi-GPU replicas design, pgmi/dist.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path.insert(0, os.path.join(repo, "multimodal-financial-analysis-tool-using-paligemma_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import types
    from pgmi.dist import broadcast_weights, gather_tokens, shard_range
    slab = torch.arange(1000, dtype=torch.uint8) if rank == 0 else torch.zeros(1000, dtype=torch.uint8)
    # an engine on the CPU: broadcast_weights takes the torch.distributed path (GPU ranks use
    # libpgmi's RCCL broadcast, pgmi_broadcast_weights) and marks the engine for re-prepare
    eng = types.SimpleNamespace(slab=slab, device=torch.device("cpu"), prepared=True)
    assert broadcast_weights(eng, src=0) is None and eng.prepared is False
    lo, hi = shard_range(64, rank, world)
    toks = torch.arange(lo, hi).reshape(-1, 1).repeat(1, 3)
    allt = gather_tokens(toks)
    q.put((rank, bool(torch.equal(slab, torch.arange(1000, dtype=torch.uint8))), allt[:, 0].tolist()))
    dist.destroy_process_group()


def test_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, ids in res:
        assert ok
        assert ids == list(range(64))


def _id_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "multimodal-financial-analysis-tool-using-paligemma_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pgmi.dist import exchange_comm_id
    uid = exchange_comm_id(torch.device("cpu"), src=0)
    q.put((rank, uid))
    dist.destroy_process_group()


def test_weight_comm_id_exchange_world2():
    """WeightComm's first half over gloo: rank 0's RCCL unique id (libpgmi -> dlopen'ed librccl,
    no GPU) reaches rank 1 byte for byte; pgmi_comm_init (a GPU call) is where the GPU path takes over."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_id_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(res[0]) == 128 and res[0] == res[1] and any(res[0])


def test_bench_dry_run_world2():
    """bench.py's N > 1 flow for real (--gpus 2 re-launches itself under torch.distributed.run as two
    gloo ranks): images sharded 8 per rank, barrier-bracketed timing with the max over ranks, every
    image's tokens gathered on rank 0, one JSON line."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "5",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 5 and out["scaling"] == "weak" and out["dry_run"]
    assert out["config"]["batch_per_gpu"] == 8 and out["config"]["global_batch"] == 16
    assert out["gathered_images"] == list(range(16)) and out["gathered_steps_ok"]
    assert out["value"] > 0
