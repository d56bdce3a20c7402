"""CPU (gloo, world_size 2): the bucketed gradient all-reduce and the
data-parallel semantics (DP gradient == mean of per-shard oracle gradients)."""
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


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "transformer-tacotron2_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def run_world(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _bucket_case(rank, world):
    from tt2.dist import GradSync
    g = torch.Generator().manual_seed(100 + rank)
    flat = torch.randn(10007, generator=g)
    expect = sum(torch.randn(10007, generator=torch.Generator().manual_seed(100 + r)) for r in range(world))
    sync = GradSync(flat, bucket_bytes=4 * 1000)
    # backward reports ready offsets in decreasing order
    for off in (9000, 8500, 5000, 4999, 100):
        sync.ready(off)
    sync.finish()
    return (flat - expect).abs().max().item()


def test_bucketed_allreduce_gloo():
    out = run_world(_bucket_case)
    assert all(v < 1e-5 for v in out.values())


def _dp_oracle_case(rank, world):
    """Each rank: oracle grads of its shard with the loss scaled by 1/world; the
    bucketed SUM then equals the mean of per-shard gradients."""
    from tt2.dist import GradSync
    from tt2_oracle import OracleConfig, TransformerTTSOracle, init_deterministic
    cfg = OracleConfig(n_enc=1, n_dec=1, d_model=64, n_heads=2, d_ffn=128, dec_prenet=32, postnet_channels=32)
    model = init_deterministic(TransformerTTSOracle(cfg), 0).train()
    shards = []
    for r in range(world):
        g = torch.Generator().manual_seed(7 + r)
        shards.append((torch.randint(1, 80, (2, 9), generator=g), torch.tensor([9, 6]),
                       torch.randn(2, 12, 80, generator=g), torch.tensor([12, 8])))

    def grads_of(shard, scale):
        model.zero_grad()
        out = model(*shard)
        loss, _ = model.loss(out[:3], shard[2], shard[3])
        (loss * scale).backward()
        return torch.cat([p.grad.reshape(-1) for p in model.parameters()])

    mine = grads_of(shards[rank], 1.0 / world).clone()
    sync = GradSync(mine, bucket_bytes=4 * 5000)
    sync.ready(mine.numel() // 2)
    sync.finish()
    ref = sum(grads_of(s, 1.0) for s in shards) / world
    return ((mine - ref).norm() / ref.norm()).item()


def test_dp_gradient_is_mean_of_shards():
    out = run_world(_dp_oracle_case)
    assert all(v < 1e-5 for v in out.values()), out


def _bnsync_case(rank, world):
    """SyncBatchNorm's exchange protocol (tt2/dist.py BnSync, the tt2_batchnorm_*_stats slot
    layout): each rank fills only its own [3][C] slot (mean, M2, row count) of the
    [world][3][C] buffer, the SUM all-reduce gives every rank every slot, and combining them
    in rank order the way bn_sync_finalize_kernel does (count-weighted mean, M2 + n_r
    (mean_r - mean)^2) gives the statistics of the concatenated rows, with ranks holding
    different row counts."""
    from tt2.dist import BnSync
    C = 16
    Ms = [37 + 11 * r for r in range(world)]
    ys = [torch.randn(Ms[r], C, generator=torch.Generator().manual_seed(50 + r), dtype=torch.float64) * (1 + r) + r
          for r in range(world)]
    s = BnSync(world, rank, device="cpu")
    buf = s.buffer((3 * world + 2) * C * 4)
    slots = buf[:world * 3 * C].view(world, 3, C)
    slots.zero_()
    y = ys[rank]
    slots[rank, 0] = y.mean(0).float()
    slots[rank, 1] = ((y - y.mean(0)) ** 2).sum(0).float()
    slots[rank, 2] = float(Ms[rank])
    s.exchange(buf[:world * 3 * C])
    n = slots[:, 2].double()
    N = n.sum(0)
    mu = (n * slots[:, 0].double()).sum(0) / N
    m2 = (slots[:, 1].double() + n * (slots[:, 0].double() - mu) ** 2).sum(0)
    full = torch.cat(ys)
    return max((mu - full.mean(0)).abs().max().item(),
               (m2 / N - full.var(0, unbiased=False)).abs().max().item() / full.var(0).max().item())


def test_syncbn_exchange_gloo():
    out = run_world(_bnsync_case)
    assert all(v < 1e-6 for v in out.values()), out


def _issue_order_case(rank, world):
    """Each rank derives its bucket issue sequence from the same ready() offsets (rank 1 also
    from a reordered copy), the sequences travel by all_gather_object, and compare_issue_logs
    must accept the identical ones and flag the reordered one at its first difference."""
    from tt2.dist import GradSync, compare_issue_logs
    sync = GradSync(torch.zeros(10007), bucket_bytes=4 * 1000)
    offs = [9000, 8500, 5000, 4999, 100]
    good = []
    for off in offs:
        good += [("bucket",) + sync.buckets[i] + ("side",) for i in sync.take_ready(off)]
    good += [("bucket",) + b + ("side",) for b in sync.buckets[sync.next:]]
    bad = list(good)
    if rank == 1:
        bad[2], bad[3] = bad[3], bad[2]   # one bucket hook fired late on rank 1
    logs_good, logs_bad = [None] * world, [None] * world
    dist.all_gather_object(logs_good, good)
    dist.all_gather_object(logs_bad, bad)
    return compare_issue_logs(logs_good), compare_issue_logs(logs_bad), good[2], good[3]


def test_compare_issue_logs_two_ranks():
    out = run_world(_issue_order_case)
    for r in range(2):
        ok, bad, b2, b3 = out[r]
        assert ok == []
        assert bad == [(1, 2, b2, b3)]


def test_compare_issue_logs_lengths():
    from tt2.dist import compare_issue_logs
    a = [("bucket", 0, 10, "side"), ("bn", 4104, "main")]
    assert compare_issue_logs([a, list(a), list(a)]) == []
    assert compare_issue_logs([a, a[:1]]) == [(1, 1, ("bn", 4104, "main"), None)]
    assert compare_issue_logs([a, a + [("bn", 1, "main")]]) == [(1, 2, None, ("bn", 1, "main"))]
    assert compare_issue_logs([a, [("bucket", 0, 10, "main"), a[1]]]) == [(1, 0, a[0], ("bucket", 0, 10, "main"))]


def test_layer_aligned_buckets():
    """Buckets cut at the backward's ready offsets (engine.ready_offsets): one bucket per reported
    range, ranges below per / 4 merged into the next lower one, covering the buffer exactly in
    reverse layout order; each bucket is complete at the ready call of its own lowest offset."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "transformer-tacotron2_amd"))
    from tt2.config import TTSConfig
    from tt2.dist import _buckets
    from tt2.params import Layout, build_slots
    cfg = TTSConfig()
    lay = Layout(build_slots(cfg))
    names = (["post.conv0.w", "heads.w"] + [f"dec{l}.qkv.w" for l in reversed(range(cfg.n_dec))] + ["dec.fc1.w"] +
             [f"enc{l}.qkv.w" for l in reversed(range(cfg.n_enc))] + ["enc.embed"])
    cuts = [lay.offset(n) for n in names]
    per = (25 << 20) // 4
    b = _buckets(lay.numel, per, cuts)
    assert b[0][1] == lay.numel and b[-1][0] == 0
    assert all(b[i][0] == b[i + 1][1] for i in range(len(b) - 1))
    assert all(lo in cuts for lo, _ in b)
    assert len(b) == 1 + cfg.n_dec + 1 + cfg.n_enc + 1          # heads merged into decoder layer 5
    assert (lay.offset("heads.w"), lay.offset("post.conv0.w")) not in b
    # fixed slices without cuts
    f = _buckets(1000, 300)
    assert f == [(700, 1000), (400, 700), (100, 400), (0, 100)]
