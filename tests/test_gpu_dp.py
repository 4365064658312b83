"""The data-parallel job driver with the real sampler: two ranks (gloo group, both on cuda:0) take a
mixed-length utterance job through parallel.run_sharded (LPT shards -> length buckets ->
CFM.sample on the HIP engine -> all-gather of the finished mels), and every rank ends with every
utterance, bit-identical to running the same batches in one process (eval_infer_batch.py:178-214
shards whole prompts per rank the same way). The reference is the same plan run sequentially, not a
world-1 plan: a batched utterance legitimately differs from the same utterance batched otherwise
(the reference says so itself, cfm.py:193-194: padded positions reach the convolutions).
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

# per job kind: (totals, refs, n_text, arch, compute, nfe, max_batch)
JOBS = {
    "tiny": ([150, 260, 190, 330, 210], [60, 100, 70, 120, 90], [30, 50, 40, 60, 45], "DiT_tiny", "fp32", 4, 2),
    # the C4 model (F5 v1 Base, bf16) on a few utterances: two ranks, one batch of two on rank 0
    "base": ([420, 300, 510], [200, 150, 260], [70, 50, 90], "F5TTS_v1_Base", "bf16", 2, 2),
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job(kind):
    from f5_tts_amd import synthetic

    totals, refs, ntext, arch = JOBS[kind][:4]
    vocab = 64 if arch == "DiT_tiny" else 2545
    utts = []
    for i, (tot, ref, nt) in enumerate(zip(totals, refs, ntext)):
        c = synthetic.make_case(B=1, ref_frames=ref, total_frames=tot, n_text=nt, seed=100 + i, vocab=vocab)
        utts.append({"cond": c["cond"][0], "text": c["text"][0][c["text"][0] >= 0], "ref": ref, "total": tot})
    return utts


def _model_and_sampler(kind):
    from f5_tts_amd import configs, synthetic
    from f5_tts_amd.model import CFM, DiT

    name, compute, nfe = JOBS[kind][3:6]
    arch = configs.get_arch(name, text_num_embeds=64) if name == "DiT_tiny" else configs.get_arch(name)
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    model = CFM(transformer=net, num_channels=100, compute=compute).to("cuda:0")

    def sample(cond, text, dur, lens):
        # one seed for every call: CFM.sample reseeds per utterance (cfm.py:196-201), so an
        # utterance's noise depends on its own duration only, not on the batch it lands in
        out, _ = model.sample(cond=cond.to("cuda:0"), text=text.to("cuda:0"), duration=dur, lens=lens, steps=nfe,
                              cfg_strength=2.0, sway_sampling_coef=-1.0, seed=0, keep_trajectory=False)
        return out.float().cpu()

    return sample


def _run(kind, rank, world):
    """The job on this rank; returns {utterance: generated mel} (CPU) for every utterance."""
    from f5_tts_amd import parallel

    return parallel.run_sharded(_job(kind), _model_and_sampler(kind), rank=rank, world=world,
                                max_batch=JOBS[kind][6], device=torch.device("cpu"))


def _sequential(kind, world):
    """Every rank's batches of the world-size plan, run one after the other in this process."""
    from f5_tts_amd import parallel

    utts, sample = _job(kind), _model_and_sampler(kind)
    plan_all = parallel.plan([u["total"] for u in utts], world, JOBS[kind][6])
    out = {}
    for r in range(world):
        out.update(parallel.run_sharded(utts, sample, rank=r, world=1, plan_all=plan_all))
    return out


def _worker(kind, rank, world, port, q):
    import sys

    sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd")]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        got = _run(kind, rank, world)
        q.put((rank, {k: v.numpy() for k, v in got.items()}))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", list(JOBS))
def test_dp_job_world2_equals_sequential_run_of_the_plan(kind):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp

    TOTALS, REFS = JOBS[kind][0], JOBS[kind][1]
    single = _sequential(kind, 2)
    assert sorted(single) == list(range(len(TOTALS)))
    for i, m in single.items():
        assert m.shape == (TOTALS[i] - REFS[i], 100) and torch.isfinite(m).all()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(kind, r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank in (0, 1):
        got = res[rank]
        assert sorted(got) == list(range(len(TOTALS))), (rank, sorted(got))
        for i, ref in single.items():
            assert torch.equal(torch.from_numpy(got[i]), ref), (rank, i)


def test_c4_rank_job_equals_direct_sample():
    """C4's per-rank workload: 32 utterances of 938 + 938 frames (300 tokens) through the job driver
    (plan -> one bucket of 32 -> CFM.sample -> generated frames) with the Base model in bf16, equal bit
    for bit to one direct CFM.sample of the same padded batch (eval_infer_batch.py:178-214 runs the
    same per-rank batches). NFE 2: the property does not depend on the step count."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from f5_tts_amd import configs, parallel, synthetic
    from f5_tts_amd.model import CFM, DiT

    arch = configs.get_arch("F5TTS_v1_Base")
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    model = CFM(transformer=net, num_channels=100, compute="bf16").to("cuda:0")
    B, ref, tot, nt = 32, 938, 1876, 300
    c = synthetic.make_case(B=B, ref_frames=ref, total_frames=tot, n_text=nt, seed=4)
    utts = [{"cond": c["cond"][i], "text": c["text"][i][c["text"][i] >= 0], "ref": ref, "total": tot} for i in range(B)]
    # the 8-GPU plan of the whole C4 job gives every rank exactly this shape of work
    plan8 = parallel.plan([tot] * 256, 8, 32)
    assert all(len(p) == 1 and len(p[0]) == 32 for p in plan8)

    def sample(cond, text, dur, lens):
        out, _ = model.sample(cond=cond.to("cuda:0"), text=text.to("cuda:0"), duration=dur, lens=lens, steps=2,
                              cfg_strength=2.0, sway_sampling_coef=-1.0, seed=0, keep_trajectory=False)
        return out

    got = parallel.run_sharded(utts, sample, rank=0, world=1, max_batch=32)
    assert sorted(got) == list(range(B))
    text = torch.nn.utils.rnn.pad_sequence([u["text"] for u in utts], batch_first=True, padding_value=-1)
    direct = sample(torch.stack([u["cond"][:ref] for u in utts]), text, torch.full((B,), tot), torch.full((B,), ref))
    torch.cuda.synchronize()
    assert direct.shape == (B, tot, 100)
    assert torch.isfinite(direct).all()
    for i in range(B):
        assert torch.equal(got[i], direct[i, ref:tot]), i
