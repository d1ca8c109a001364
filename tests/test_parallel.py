"""Multi-rank paths of hyperopt_amd.parallel.

CPU (gloo, world_size 2): candidate sharding covers [0, n) exactly once, the
all-gather lays records out as [world][S][P], and merging per-rank winners
with numpy argmax semantics reproduces the unsharded np.argmax (ties, NaN,
inactive hps).  GPU: two gloo ranks on one MI355X run ShardedSuggest on a
conditional space and must equal the unsharded device suggest."""
import os
import socket
import tempfile

import numpy as np
import pytest

from hyperopt_amd import parallel as PAR
from hyperopt_amd._engine import RESULT_DTYPE


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(fn, world, *args):
    import torch.multiprocessing as mp
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(fn, args=(world, port, d) + args, nprocs=world, join=True)
        return [np.load(os.path.join(d, 'r%d.npy' % r), allow_pickle=False)
                for r in range(world)]


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    return dist


@pytest.mark.parametrize('n', [0, 1, 7, 24, 4096, 10_000_019])
@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_shard_range_partitions(n, world):
    spans = [PAR.shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0
    for (b0, c0), (b1, _) in zip(spans, spans[1:]):
        assert b0 + c0 == b1
    assert sum(c for _, c in spans) == n
    assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    assert list(PAR.suggestion_slice(10, 1, 4)) == [3, 4, 5]
    with pytest.raises(ValueError):
        PAR.shard_range(n, world, world)


@pytest.mark.parametrize('n', [0, 1, 4095, 4096, 5000, 1 << 22, 10_000_000])
@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_shard_range_aligned(n, world):
    """Boundaries at multiples of the sorted-draw block (TPE_SHARD_ALIGN):
    the shards' bucketed blocks are the unsharded suggest's blocks."""
    from hyperopt_amd._engine import SHARD_ALIGN as A
    spans = [PAR.shard_range(n, r, world, A) for r in range(world)]
    assert spans[0][0] == 0 and sum(c for _, c in spans) == n
    for (b0, c0), (b1, _) in zip(spans, spans[1:]):
        assert b0 + c0 == b1 and b1 % A == 0 or b1 == n
    full = [c for _, c in spans if c % A == 0 or _ + c == n]
    assert len(full) == world
    units = [-(-c // A) for _, c in spans]
    assert max(units) - min(units) <= 1


def _scores(S, P, n, seed):
    """Synthetic per-candidate EI scores with ties, NaN and -inf, and an
    inactive hp (index -1 everywhere)."""
    rng = np.random.RandomState(seed)
    sc = np.round(rng.randn(S, P, n), 1)          # many exact ties
    sc[0, 1, rng.randint(n, size=3)] = np.nan      # NaN wins at first index
    sc[1 % S, 2, :] = -np.inf
    return sc


def _local_records(sc, begin, count, inactive_hp):
    S, P, _ = sc.shape
    rec = np.zeros((S, P), dtype=RESULT_DTYPE)
    for s in range(S):
        for p in range(P):
            if p == inactive_hp:
                rec[s, p] = (np.nan, np.nan, -1, 0, 0)
                continue
            part = sc[s, p, begin:begin + count]
            if count == 0:
                rec[s, p] = (np.nan, np.nan, -1, 1, 0)
                continue
            i = int(np.argmax(part))
            rec[s, p] = (part[i], 1000.0 + begin + i, begin + i, 1, 0)
    return rec


def _gather_worker(rank, world, port, outdir, S, P, n):
    import torch
    _init(rank, world, port)
    sc = _scores(S, P, n, 0)
    b, c = PAR.shard_range(n, rank, world)
    rec = _local_records(sc, b, c, inactive_hp=3)
    local = torch.from_numpy(rec.view(np.uint8).reshape(-1).copy())
    g = PAR.gather_records(local)
    np.save(os.path.join(outdir, 'r%d.npy' % rank), g.numpy())
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.parametrize('world,n', [(2, 97), (2, 1), (3, 50)])
def test_gloo_gather_and_merge_equal_unsharded_argmax(world, n):
    S, P = 2, 4
    outs = _spawn(_gather_worker, world, S, P, n)
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])         # every rank sees the same
    g = outs[0].view(RESULT_DTYPE).reshape(world, S, P)  # [world][S][P]
    merged = PAR.merge_records_host(g)
    sc = _scores(S, P, n, 0)
    for s in range(S):
        for p in range(P):
            r = merged[s, p]
            if p == 3:
                assert r['active'] == 0 and r['index'] == -1
                continue
            want = int(np.argmax(sc[s, p]))
            assert r['index'] == want, (s, p, r, want)
            assert r['value'] == 1000.0 + want
            assert r['active'] == 1


def test_merge_prefers_first_nan_and_lowest_tied_index():
    rec = np.zeros((3, 1, 1), dtype=RESULT_DTYPE)
    rec[0, 0, 0] = (2.0, 0.5, 40, 1, 0)
    rec[1, 0, 0] = (2.0, 0.7, 10, 1, 0)   # tie -> lower global index
    rec[2, 0, 0] = (1.0, 0.9, 99, 1, 0)
    assert PAR.merge_records_host(rec)[0, 0]['index'] == 10
    rec[2, 0, 0] = (np.nan, 0.9, 99, 1, 0)
    assert PAR.merge_records_host(rec)[0, 0]['index'] == 99
    rec[0, 0, 0] = (np.nan, 0.5, 40, 1, 0)
    assert PAR.merge_records_host(rec)[0, 0]['index'] == 40


# ---------------------------------------------------------------- GPU
def _gpu_worker(rank, world, port, outdir, n_cand):
    import torch
    import torch.distributed as dist
    import hyperopt_amd as H
    from hyperopt_amd import hp, rand, Trials, trials_from_docs, _engine as E
    from hyperopt_amd.base import Domain
    from hyperopt_amd.tpe import build_history
    import spaces
    _init(rank, world, port)
    torch.cuda.set_device(0)
    dom = Domain(lambda x: 0.0, spaces.cond_space(hp))
    docs = rand.suggest(list(range(300)), dom, Trials(), 3)
    for d, l in zip(docs, np.random.RandomState(4).rand(300)):
        d['state'] = H.JOB_STATE_DONE
        d['result'] = {'status': 'ok', 'loss': float(l)}
    _, losses, vals, act = build_history(dom, trials_from_docs(docs), dom.space.labels)
    hps, conds, pprior = dom.space.engine_tables()
    eng = E.Engine(0)
    plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    sh = PAR.ShardedSuggest(plan)
    sh.fit()  # on the sharded stream: ordered before its suggest
    sharded = sh.suggest([5, 6, 7], n_cand)
    if rank == 0:
        full = plan.suggest([5, 6, 7], n_cand)
        np.save(os.path.join(outdir, 'full.npy'), full.view(np.uint8))
    np.save(os.path.join(outdir, 'r%d.npy' % rank), sharded.view(np.uint8))
    torch.cuda.synchronize()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize('n_cand', [10000, 24, 4096])
def test_sharded_suggest_two_ranks_equals_single_device(n_cand):
    """Two ranks on one GPU equal one device.  24 and 4096 candidates leave
    rank 1 an empty shard (8192-aligned shards): its records must say
    "nothing here" (NaN, -1, inactive) and not leak a previous suggest's
    winners into the merge (tpe.py:750-759: no samples, no value)."""
    import torch.multiprocessing as mp
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gpu_worker, args=(2, port, d, n_cand), nprocs=2, join=True)
        full = np.load(os.path.join(d, 'full.npy')).view(RESULT_DTYPE)
        for r in range(2):
            got = np.load(os.path.join(d, 'r%d.npy' % r)).view(RESULT_DTYPE)
            np.testing.assert_array_equal(got['active'], full['active'])
            np.testing.assert_array_equal(got['index'], full['index'])
            np.testing.assert_array_equal(got['value'], full['value'])


def _gpu_worker_cfg4(rank, world, port, outdir, n_cand):
    """Config 4 (100-D, N = 1e4, K_a ~ 9976) sharded over the ranks, as
    bench.py --config cfg4 --gpus N runs it (bucketed draws, block skip)."""
    import torch
    import torch.distributed as dist
    from hyperopt_amd import hp, _engine as E
    from hyperopt_amd.base import Domain
    import big_configs
    _init(rank, world, port)
    torch.cuda.set_device(0)
    dom, losses, vals, act = big_configs.cfg4_domain_history(hp, Domain)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.Engine(0), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    sh = PAR.ShardedSuggest(plan)
    sh.fit()  # on the sharded stream: ordered before its suggest
    sharded = sh.suggest([7], n_cand)
    if rank == 0:
        full = plan.suggest([7], n_cand)
        np.save(os.path.join(outdir, 'full.npy'), full.view(np.uint8))
    np.save(os.path.join(outdir, 'r%d.npy' % rank), sharded.view(np.uint8))
    torch.cuda.synchronize()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_config4_two_ranks_equals_single_device():
    """bench.py's multi-GPU config-4 mode on one GPU with two ranks: the
    all-gathered, device-merged winners of every hp equal one device's byte
    for byte (shards aligned to TPE_SHARD_ALIGN: the same bucketed blocks,
    the same pruned / one-exponent sums)."""
    import torch.multiprocessing as mp
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gpu_worker_cfg4, args=(2, port, d, 1 << 22), nprocs=2, join=True)
        full = np.load(os.path.join(d, 'full.npy')).view(RESULT_DTYPE)
        assert (full['active'] == 1).all() and (full['index'] >= 0).all()
        for r in range(2):
            got = np.load(os.path.join(d, 'r%d.npy' % r)).view(RESULT_DTYPE)
            np.testing.assert_array_equal(got.view(np.uint8), full.view(np.uint8),
                                          err_msg='rank %d' % r)


def _nccl_worker(rank, world, port, outdir):
    """One rank over RCCL (backend 'nccl'): ShardedSuggest's gather takes the
    all_gather_into_tensor branch on device memory."""
    import torch
    import torch.distributed as dist
    import hyperopt_amd as H
    from hyperopt_amd import hp, rand, Trials, trials_from_docs, _engine as E
    from hyperopt_amd.base import Domain
    from hyperopt_amd.tpe import build_history
    import spaces
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=rank, world_size=world,
                            device_id=torch.device('cuda', 0))
    dom = Domain(lambda x: 0.0, spaces.cond_space(hp))
    docs = rand.suggest(list(range(300)), dom, Trials(), 3)
    for d, l in zip(docs, np.random.RandomState(4).rand(300)):
        d['state'] = H.JOB_STATE_DONE
        d['result'] = {'status': 'ok', 'loss': float(l)}
    _, losses, vals, act = build_history(dom, trials_from_docs(docs), dom.space.labels)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.Engine(0), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    assert dist.get_backend() == 'nccl'
    sh = PAR.ShardedSuggest(plan)
    sh.fit()
    got = sh.suggest([5, 6], 3000)
    full = plan.suggest([5, 6], 3000)
    np.save(os.path.join(outdir, 'got.npy'), got.view(np.uint8))
    np.save(os.path.join(outdir, 'full.npy'), full.view(np.uint8))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_suggest_over_rccl_one_rank():
    import torch.multiprocessing as mp
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_nccl_worker, args=(1, port, d), nprocs=1, join=True)
        got = np.load(os.path.join(d, 'got.npy'))
        np.testing.assert_array_equal(got, np.load(os.path.join(d, 'full.npy')))
