"""Multi-process (gloo, world_size 2) coverage of the data-parallel path: LPT sharding, length
bucketing and the all-gather of finished mels (the only collective on the sampling path)."""

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from f5_tts_amd import parallel, synthetic


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_lpt_balances_quadratic_cost():
    c3 = synthetic.c3_case()
    frames = c3["total"]
    shards = parallel.shard_lpt(frames, 8)
    assert sorted(i for s in shards for i in s) == list(range(len(frames)))
    loads = [sum(parallel.utterance_cost(frames[i]) for i in s) for s in shards]
    assert max(loads) / min(loads) < 1.15
    # count-based split (what split_between_processes does) is worse for ragged lengths
    naive = [list(range(r * 4, r * 4 + 4)) for r in range(8)]
    nl = [sum(parallel.utterance_cost(frames[i]) for i in s) for s in naive]
    assert max(loads) < max(nl)


def test_bucket_keeps_neighbours():
    frames = [100, 900, 300, 500, 700, 200]
    b = parallel.bucket(range(6), frames, 2)
    assert [[frames[i] for i in x] for x in b] == [[100, 200], [300, 500], [700, 900]]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = [120, 80, 200, 50, 160]
    shards = parallel.shard_lpt(frames, world)
    # stand-in for the engine's output: a deterministic mel per utterance
    local = {i: torch.full((frames[i], 100), float(i)) + torch.arange(frames[i])[:, None] for i in shards[rank]}
    got = parallel.gather_mels(local)
    ok = sorted(got) == list(range(len(frames))) and all(
        torch.equal(got[i], torch.full((frames[i], 100), float(i)) + torch.arange(frames[i])[:, None])
        for i in range(len(frames)))
    q.put((rank, ok, [len(s) for s in shards]))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_mels_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(p.exitcode == 0 for p in procs)


def _fake_sample(cond, text, duration, lens):
    """Deterministic stand-in for CFM.sample: row n of utterance b is a function of its own inputs
    only (prompt sum, token sum, lengths, position), so a misrouted or duplicated result shows."""
    B, N = cond.shape[0], int(duration.max())
    out = torch.zeros(B, N, 100)
    for b in range(B):
        tok = float(text[b][text[b] >= 0].sum())
        base = float(cond[b, : int(lens[b])].sum()) + tok + 1000.0 * float(duration[b])
        out[b, : int(duration[b])] = base + torch.arange(int(duration[b]))[:, None] * 0.5 + torch.arange(100)[None]
    return out


def _job(n=11):
    g = torch.Generator().manual_seed(3)
    utts = []
    for i in range(n):
        total = int(torch.randint(60, 400, (1,), generator=g))
        ref = total // 3
        utts.append(dict(cond=torch.randn(ref, 100, generator=g), text=torch.randint(0, 50, (ref // 4 + 1,), generator=g),
                         ref=ref, total=total))
    return utts


def _expected(u):
    cond = u["cond"][None]
    return _fake_sample(cond, u["text"][None], torch.tensor([u["total"]]), torch.tensor([u["ref"]]))[0, u["ref"]:u["total"]]


def _job_worker(rank, world, port, q, n=11):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    utts = _job(n)
    calls = []

    def sample(cond, text, dur, lens):
        calls.append(len(dur))
        return _fake_sample(cond, text, dur, lens)

    got = parallel.run_sharded(utts, sample, rank=rank, world=world, max_batch=3)
    ok = sorted(got) == list(range(len(utts))) and all(torch.equal(got[i], _expected(utts[i])) for i in got)
    q.put((rank, ok, calls))
    dist.barrier()
    dist.destroy_process_group()


def test_run_sharded_world2_gloo_every_utterance_once():
    """The DP job driver end to end (eval_infer_batch.py:178-214 pattern): 11 mixed-length utterances,
    LPT over 2 ranks, buckets of at most 3, an injected stand-in sampler; every rank ends with every
    utterance exactly once, each equal to the stand-in's single-utterance result, and the two ranks
    together sampled every utterance exactly once."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_job_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert sum(sum(c) for _, _, c in res) == 11
    assert all(max(c) <= 3 for _, _, c in res)
    assert all(p.exitcode == 0 for p in procs)


def test_run_sharded_world2_one_utterance_empty_rank():
    """Fewer utterances than ranks: the rank holding none still joins the layout all-gather (CPU
    device, channel count from the job) and ends with the one utterance."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_job_worker, args=(r, 2, port, q, 1)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert sorted(sum(c) for _, _, c in res) == [0, 1]
    assert all(p.exitcode == 0 for p in procs)


def test_run_sharded_world1_no_collective():
    utts = _job(5)
    got = parallel.run_sharded(utts, _fake_sample, rank=0, world=1, max_batch=2)
    assert sorted(got) == list(range(5))
    for i, u in enumerate(utts):
        assert torch.equal(got[i], _expected(u))

