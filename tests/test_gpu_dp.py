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

TOTALS = [150, 260, 190, 330, 210]
REFS = [60, 100, 70, 120, 90]
NTEXT = [30, 50, 40, 60, 45]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job():
    from f5_tts_amd import synthetic

    utts = []
    for i, (tot, ref, nt) in enumerate(zip(TOTALS, REFS, NTEXT)):
        c = synthetic.make_case(B=1, ref_frames=ref, total_frames=tot, n_text=nt, seed=100 + i, vocab=64)
        utts.append({"cond": c["cond"][0], "text": c["text"][0][c["text"][0] >= 0], "ref": ref, "total": tot})
    return utts


def _model_and_sampler():
    from f5_tts_amd import configs, synthetic
    from f5_tts_amd.model import CFM, DiT

    arch = configs.get_arch("DiT_tiny", text_num_embeds=64)
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    model = CFM(transformer=net, num_channels=100, compute="fp32").to("cuda:0")

    def sample(cond, text, dur, lens):
        # one seed for every call: CFM.sample reseeds per utterance (cfm.py:196-201), so an
        # utterance's noise depends on its own duration only, not on the batch it lands in
        out, _ = model.sample(cond=cond.to("cuda:0"), text=text.to("cuda:0"), duration=dur, lens=lens, steps=4,
                              cfg_strength=2.0, sway_sampling_coef=-1.0, seed=0, keep_trajectory=False)
        return out.cpu()

    return sample


def _run(rank, world):
    """The job on this rank; returns {utterance: generated mel} (CPU) for every utterance."""
    from f5_tts_amd import parallel

    return parallel.run_sharded(_job(), _model_and_sampler(), rank=rank, world=world, max_batch=2,
                                device=torch.device("cpu"))


def _sequential(world):
    """Every rank's batches of the world-size plan, run one after the other in this process."""
    from f5_tts_amd import parallel

    utts, sample = _job(), _model_and_sampler()
    plan_all = parallel.plan([u["total"] for u in utts], world, 2)
    out = {}
    for r in range(world):
        out.update(parallel.run_sharded(utts, sample, rank=r, world=1, plan_all=plan_all))
    return out


def _worker(rank, world, port, q):
    import sys

    sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd")]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        got = _run(rank, world)
        q.put((rank, {k: v.numpy() for k, v in got.items()}))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_dp_job_world2_equals_sequential_run_of_the_plan():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp

    single = _sequential(2)
    assert sorted(single) == list(range(len(TOTALS)))
    for i, m in single.items():
        assert m.shape == (TOTALS[i] - REFS[i], 100) and torch.isfinite(m).all()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
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
