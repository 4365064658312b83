"""Data-parallel sharding of utterances over GPUs.

The sampling path never communicates inside the ODE: each rank runs the engine on its own
utterances. This module holds the two host-side pieces around that:

* `shard_lpt`: longest-processing-time assignment of utterances to ranks by the cost model
  S*F(N) with F(N) = a*N + b*N^2, the MI355X replacement for the reference's
  `split_between_processes` (eval_infer_batch.py:181) / `DistributedSampler`
  (benchmark.py:340-341), which split by count and ignore the quadratic attention term.
* `gather_mels`: the only collective on the path — an all-gather of per-rank counts and
  lengths, then of the finished mels (padded to the max per rank), over RCCL (backend
  "nccl") on GPUs or gloo on CPU.
* `run_sharded`: the job driver that strings them together the way the reference's eval driver
  does (eval_infer_batch.py:178-214: barrier, split the prompts over processes, per batch
  `model.sample(cond, text, duration, lens, ...)`, keep `gen[ref_len:total_len]`, barrier), with
  LPT sharding and length buckets instead of a count split, and the finished mels gathered to
  every rank instead of written to per-utterance files.
"""

from __future__ import annotations

import heapq

import torch
import torch.distributed as dist

# Base DiT: FLOPs per sequence-forward = A*N + B*N^2
COST_A, COST_B = 378.888e6, 90112.0


def utterance_cost(n_frames: int) -> float:
    return COST_A * n_frames + COST_B * n_frames * n_frames


def shard_lpt(frames, world: int):
    """Assign utterance indices to `world` ranks, heaviest first onto the least-loaded rank.
    Returns a list (per rank) of index lists, each sorted by length (for length bucketing)."""
    order = sorted(range(len(frames)), key=lambda i: -utterance_cost(frames[i]))
    heap = [(0.0, r) for r in range(world)]
    out = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + utterance_cost(frames[i]), r))
    return [sorted(o, key=lambda i: frames[i]) for o in out]


def bucket(indices, frames, max_batch: int):
    """Split a rank's (length-sorted) utterances into batches of at most `max_batch`
    (neighbours in length -> little padding, as get_inference_prompt's buckets do)."""
    idx = sorted(indices, key=lambda i: frames[i])
    return [idx[k:k + max_batch] for k in range(0, len(idx), max_batch)]


def gather_mels(local: "dict[int, torch.Tensor]", device=None, group=None, layout=None, num_channels=None):
    """All-gather finished mels {utt_index: [n_i, C]} from every rank.
    Returns {utt_index: tensor} with every utterance of the job (on every rank).

    layout: per rank, the [(utt_index, n_frames), ...] it holds, when every rank knows the plan
    (run_sharded does): then only the padded mel buffers travel and no count or index is read back
    to the host, so the gather never waits for the device. A rank may hold no utterance (fewer
    utterances than ranks): its buffer is then all padding, on `device` (CPU when not given), with
    `num_channels` channels (default: the local mels', else 100)."""
    world = dist.get_world_size(group)
    if layout is not None:
        if device is not None:
            dev = device
        else:
            dev = next(iter(local.values())).device if local else torch.device("cpu")
        C = num_channels if num_channels is not None else (next(iter(local.values())).shape[-1] if local else 100)
        maxn = max(len(x) for x in layout)
        maxl = max((n for x in layout for _, n in x), default=0)
        buf = torch.zeros(maxn, maxl, C, dtype=torch.float32, device=dev)
        for j, (k, n) in enumerate(layout[dist.get_rank(group)]):
            buf[j, :n] = local[k].float()
        bufs = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(bufs, buf, group=group)
        return {k: bufs[r][j, :n] for r in range(world) for j, (k, n) in enumerate(layout[r])}
    dev = device if device is not None else (next(iter(local.values())).device if local else torch.device("cpu"))
    C = num_channels if num_channels is not None else (next(iter(local.values())).shape[-1] if local else 100)
    keys = sorted(local)
    cnt = torch.tensor([len(keys), max([local[k].shape[0] for k in keys], default=0)], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    maxn = max(int(c[0]) for c in cnts)
    maxl = max(int(c[1]) for c in cnts)
    meta = torch.full((maxn, 2), -1, dtype=torch.int64, device=dev)
    buf = torch.zeros(maxn, maxl, C, dtype=torch.float32, device=dev)
    for j, k in enumerate(keys):
        meta[j, 0], meta[j, 1] = k, local[k].shape[0]
        buf[j, : local[k].shape[0]] = local[k].float()
    metas = [torch.empty_like(meta) for _ in range(world)]
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    dist.all_gather(bufs, buf, group=group)
    out = {}
    for m, b in zip(metas, bufs):
        for j in range(maxn):
            k, n = int(m[j, 0]), int(m[j, 1])
            if k >= 0:
                out[k] = b[j, :n].clone()
    return out


def padded_mel_batch(mels, length=None):
    """[n_i, C] mels -> [B, max n_i (or length), C], zero padded (utils_eval.py:58-66, frame-major)."""
    n = max(m.shape[0] for m in mels) if length is None else length
    out = mels[0].new_zeros(len(mels), n, mels[0].shape[-1])
    for i, m in enumerate(mels):
        out[i, : m.shape[0]] = m
    return out


def plan(totals, world: int, max_batch: int):
    """Per rank, the list of batches (utterance index lists): LPT over ranks, then length buckets."""
    return [bucket(idx, totals, max_batch) for idx in shard_lpt(totals, world)]


def run_sharded(utts, sample_fn, *, rank: int, world: int, max_batch: int = 32, device=None, group=None,
                plan_all=None):
    """Run a whole utterance job data-parallel and return {index: generated mel [total-ref, C]} on
    every rank.

    utts: list of dicts with `cond` [ref_i(, padded), C] mel, `text` (str list or id list), `ref` (prompt
    frames) and `total` (total frames), the fields of one prompt in eval_infer_batch.py:182-185.
    sample_fn(cond [B,Nc,C], text list, duration LongTensor[B], lens LongTensor[B]) -> out [B,N,C]: the
    engine's `CFM.sample` (or a stand-in in tests). `plan_all` (from `plan`, every rank's batches) may be
    passed to reuse a plan across calls. World 1 runs without any collective."""
    if plan_all is None:
        plan_all = plan([u["total"] for u in utts], world, max_batch)
    batches = plan_all[rank]
    local = {}
    for b in batches:
        cond = padded_mel_batch([utts[i]["cond"][: utts[i]["ref"]] for i in b])
        if device is not None:
            cond = cond.to(device)
        text = [utts[i]["text"] for i in b]
        if torch.is_tensor(text[0]):  # token ids: one [B, nt] LongTensor, -1 padded (list_str_to_idx layout)
            text = torch.nn.utils.rnn.pad_sequence(text, batch_first=True, padding_value=-1)
        # lengths stay host tensors: CFM.sample evaluates its duration rule on the host without a sync
        dur = torch.tensor([utts[i]["total"] for i in b], dtype=torch.long)
        lens = torch.tensor([utts[i]["ref"] for i in b], dtype=torch.long)
        out = sample_fn(cond, text, dur, lens)
        for j, i in enumerate(b):
            local[i] = out[j, utts[i]["ref"]: utts[i]["total"]]
    if world == 1:
        return local
    layout = [[(i, utts[i]["total"] - utts[i]["ref"]) for b in plan_all[r] for i in b] for r in range(world)]
    return gather_mels(local, device=device, group=group, layout=layout, num_channels=utts[0]["cond"].shape[-1])

