"""N > 1 path on CPU: world-size-2 gloo run of the shard / argmin-gather logic
(apf_quadruped_amd/shard.py) that bench.py uses with RCCL on the GPUs.

Each rank solves its own contiguous shard (here with the oracle, the CPU
checker), reduces it to (fval, local index) with the qpb_argmin rule, and the
ranks exchange their payload (fval, local index, x*[12]: 16 + 96 B each, as
qpb_winner builds it on the GPU); the gathered winner and its x* must equal the
single-process argmin over the whole batch."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

PER_RANK = 12
SEED = 0xD06B07 + 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve_fvals(ids):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_py import Oracle
    from apf_quadruped_amd import workloads as W
    o = Oracle()
    d = W.contact_force_qp(SEED, ids)
    Pc, Ac, Gc = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    fv, fl, xs = [], [], []
    for k in range(len(ids)):
        r = o.solve_dense(12, 20, 6, Pc[k], Ac[k], Gc[k], d["c"][k], d["h"][k], d["b"][k])
        fv.append(r["fval"])
        fl.append(r["flag"])
        xs.append(r["x"])
    return np.array(fv), np.array(fl), np.array(xs)


def _local_argmin(fv, fl):
    best = (np.inf, -1)
    for i, (v, f) in enumerate(zip(fv, fl)):
        if f == 0 and (best[1] < 0 or v < best[0]):
            best = (v, i)
    return best


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from apf_quadruped_amd.shard import all_gather_winner, global_winner, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(rank, world, PER_RANK)
    fv, fl, xs = _solve_fvals(np.arange(lo, hi))
    v, i = _local_argmin(fv, fl)
    payload = np.concatenate([[v, float(i)], xs[i] if i >= 0 else np.full(12, np.nan)])
    g = all_gather_winner(torch.tensor(payload, dtype=torch.float64), world)
    offsets = [shard_range(r, world, PER_RANK)[0] for r in range(world)]
    wv, wi, wr = global_winner(g.numpy(), offsets, width=14)
    q.put((rank, (wv, wi, wr, g.numpy()[wr, 2:].tolist())))
    dist.destroy_process_group()


def test_two_rank_gloo_argmin_gather():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fv, fl, xs = _solve_fvals(np.arange(world * PER_RANK))
    v, i = _local_argmin(fv, fl)
    for r in range(world):
        assert res[r][0] == v and res[r][1] == i, (r, res[r], (v, i))
        np.testing.assert_array_equal(res[r][3], xs[i])          # every rank holds the winner's x*


def test_shard_helpers():
    from apf_quadruped_amd.shard import global_winner, shard_range, split_even
    assert shard_range(3, 8, 8192) == (24576, 32768)
    assert [split_even(10, 3, r) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    with pytest.raises(ValueError):
        shard_range(2, 2, 1)
    # ties -> lowest global index; ranks without an optimal QP (-1) are skipped
    g = [[1.0, 5], [1.0, 0], [np.inf, -1]]
    assert global_winner(g, [0, 100, 200]) == (1.0, 5, 0)
    assert global_winner([[np.inf, -1]], [0]) == (np.inf, -1, -1)


def _comm_worker(rank, world, port, q):
    import torch.distributed as dist
    from apf_quadruped_amd.shard import ArgminGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ArgminGather(rank, world)
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, f"raised: {e}"))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_comm_setup_fails_on_every_rank_without_a_gpu():
    """ArgminGather's bootstrap (rank 0 makes the RCCL unique id, every rank gets it
    by broadcast, then every rank joins the communicator) must fail on every rank
    alike without a GPU -- whether rank 0 cannot make the id (the error travels in
    the broadcast) or the communicator cannot be made -- so bench.py's fallback is
    collective and no rank waits forever."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(v.startswith("raised") for v in res.values()), res


def _agree_worker(rank, world, port, q):
    import torch.distributed as dist
    from apf_quadruped_amd.shard import TorchGather, make_argmin_gather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ag, info = make_argmin_gather(rank, world, "cpu")
    q.put((rank, (isinstance(ag, TorchGather), info["gather"], info["rccl_ranks"], bool(info["init_error"]))))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_path_is_agreed_on_every_rank():
    """bench.py's gather path (make_argmin_gather): when the RCCL communicator cannot
    be made, EVERY rank falls back to the torch gather (the ranks all_reduce the init
    outcome), and the bench line records which path ran."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] == (True, "torch_fallback", None, True), res


def _bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    """`bench.py --gpus N` (no torchrun) starts N rank processes itself, each with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, which join one process group
    (gloo in --dry-run, which stops before the first GPU call) and own contiguous
    shards; rank 0 prints the one line with n_gpus == N."""
    rc, line, err = _bench(["--gpus", str(n), "--batch", "8192", "--dry-run"])
    assert rc == 0, err
    assert line["n_gpus"] == n and line["gpus_arg"] == n
    assert [(d["rank"], d["local_rank"], d["world"]) for d in line["ranks"]] == [(r, r, n) for r in range(n)]
    assert [(d["lo"], d["hi"]) for d in line["ranks"]] == [(r * 8192, (r + 1) * 8192) for r in range(n)]
    assert line["master"][0] == "127.0.0.1"


def test_bench_launcher_parent_never_loads_hip(tmp_path):
    """The `--gpus N` launcher process itself loads no HIP runtime and does not import
    torch (its device count comes from a throwaway child): checked from the parent's
    own /proc/self/maps after its ranks have run."""
    maps = tmp_path / "maps.json"
    rc, line, err = _bench(["--gpus", "2", "--batch", "1024", "--dry-run"], {"QPB_BENCH_PARENT_MAPS": str(maps)})
    assert rc == 0, err
    rep = json.loads(maps.read_text())
    assert rep["libs"], "no shared objects read from /proc/self/maps"
    assert not rep["torch_imported"]
    bad = [lib for lib in rep["libs"] if "amdhip" in lib or "hsa-runtime" in lib or "libtorch" in lib
           or "rccl" in lib]
    assert not bad, bad


def test_bench_refuses_rank_count_mismatch():
    """Under an external launcher, --gpus must equal WORLD_SIZE: the bench never
    measures another rank count than the one asked for."""
    rc, line, err = _bench(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and line is None and "WORLD_SIZE=2" in err


def test_bench_refuses_missing_gpus():
    """Without --dry-run, --gpus N on a machine with fewer than N GPUs exits
    non-zero before starting any rank (no silent fallback to fewer ranks)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this machine has two GPUs")
    rc, line, err = _bench(["--gpus", "2"])
    assert rc == 2 and line is None and "needs 2 visible GPUs" in err
