"""Fused Adam + global-norm clip + Noam LR vs an independent
implementation: torch.optim.Adam / AdamW + torch.nn.utils.clip_grad_norm_ + LambdaLR(Noam)
in float64 on the CPU, three steps over a random flat buffer (the third with a gradient
norm below the clip, so no clipping).  Parameters, both moments and the bf16 shadow must
agree to 1e-6 relative (the parameter update itself to 1e-5)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def noam(step, d_model, warmup):
    return d_model ** -0.5 * min(step ** -0.5, step * warmup ** -1.5)


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_adam_clip_noam_matches_torch(wd):
    n = 65536 + 48                 # flat slots are 16-aligned; exercises the float4 body only
    d_model, warmup, clip, lr = 512, 4.0, 1.0, 1.0
    g = torch.Generator().manual_seed(11)
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * s for s in (0.5, 2.0, 1e-4)]   # norms ~128, ~512, ~0.03

    ref = torch.nn.Parameter(p0.double().clone())
    opt_cls = torch.optim.AdamW if wd > 0 else torch.optim.Adam
    opt = opt_cls([ref], lr=lr, betas=(0.9, 0.98), eps=1e-9, weight_decay=wd)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda e: noam(e + 1, d_model, warmup))

    p = p0.cuda()
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    shadow = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    step = torch.zeros(1, dtype=torch.int32, device="cuda")
    for gr in grads:
        ref.grad = gr.double().clone()
        torch.nn.utils.clip_grad_norm_([ref], clip)
        opt.step()
        sched.step()
        ops.adam_step(p, gr.cuda(), m, v, shadow, step, n, lr, beta1=0.9, beta2=0.98, eps=1e-9, weight_decay=wd,
                      clip_norm=clip, warmup=warmup, noam=True, d_model=d_model)
        ops.step_bump(step)
        st = opt.state[ref]
        assert rel(p, ref.detach()) < 1e-6
        assert rel(p - p0.cuda(), ref.detach() - p0.double()) < 1e-5
        assert rel(m, st["exp_avg"]) < 1e-6
        assert rel(v, st["exp_avg_sq"]) < 1e-6
        assert torch.equal(shadow, p.bfloat16())
    assert step.item() == 3
