"""DDPM sampling on the GPU: Diffusion.p_sample / Diffusion.sample (model.py:167-194)
as driven by inference.py:225-230 — F = 1 forwards, fused update kernel, HIP-graph replay per step.

* cesm_ddpm_step vs the reference's eager torch expression on the same device (same operation order,
  no contraction: agreement to fp32 rounding, rtol 2e-6);
* graph-replayed sampling == the eager p_sample loop (same kernels, same RNG draws) — exact;
* fp32 sampling vs the CPU oracle's loop (oracle/ref_cpu.py Diffusion.sample) on identical x_T and step
  noises: relative L2 < 1e-4 after all steps (per-step forward parity is 1e-5; the update is linear).
"""
import pytest
import torch

from cesm_emulator_amd import kernels as K
from cesm_emulator_amd.model import UNet, Diffusion
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b).clamp_min(1e-30)).item()


def test_ddpm_step_matches_reference_expression(dev):
    d = Diffusion(UNet(ch_mults=(1, 2, 4))).to(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    B, H, W = 3, 17, 29
    x = torch.randn(B, 1, H, W, device=dev, generator=g)
    eps = torch.randn_like(x)
    z = torch.randn_like(x)
    for tv in ([999, 500, 1], [0, 0, 0], [0, 7, 999]):
        t = torch.tensor(tv, device=dev)
        b = d.betas[t].view(-1, 1, 1, 1)
        s1 = d.sqrt_one_minus_alphas_cumprod[t].view(-1, 1, 1, 1)
        r = d.sqrt_recip_alphas[t].view(-1, 1, 1, 1)
        mean = r * (x - b / s1 * eps)
        ref = mean + torch.sqrt(d.posterior_variance[t].view(-1, 1, 1, 1)) * z
        out = K.ddpm_step(x, eps, z, t, *d._coefs())
        print(tv, "max |diff|", (out - ref).abs().max().item())
        assert torch.allclose(out, ref, rtol=2e-6, atol=1e-7), tv
        assert torch.allclose(K.ddpm_step(x, eps, None, t, *d._coefs()), mean, rtol=2e-6, atol=1e-7), tv
    # in place (out aliases x)
    t = torch.tensor([5, 6, 7], device=dev)
    ref = K.ddpm_step(x, eps, z, t, *d._coefs())
    xi = x.clone()
    K.ddpm_step(xi, eps, z, t, *d._coefs(), out=xi)
    assert torch.equal(xi, ref)


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
def test_graph_sampler_equals_eager(dev, cdt):
    torch.manual_seed(1)
    net = UNet(ch_mults=(1, 2, 4)).to(dev)
    net.compute_dtype = cdt
    d = Diffusion(net, timesteps=12).to(dev)
    cond = torch.randn(2, 1, 16, 24, device=dev)
    torch.manual_seed(7)
    torch.cuda.manual_seed(7)
    y_eager = d.sample(cond, (2, 1, 16, 24), dev, use_graph=False)
    torch.manual_seed(7)
    torch.cuda.manual_seed(7)
    y_graph = d.sample(cond, (2, 1, 16, 24), dev, use_graph=True)
    assert torch.isfinite(y_graph).all()
    assert torch.equal(y_graph, y_eager)


def test_sampler_matches_oracle_fp32(dev):
    torch.manual_seed(1)
    ref = R.UNet(ch_mults=(1, 2, 4))
    torch.manual_seed(1)
    prod = UNet(ch_mults=(1, 2, 4))
    prod.load_state_dict(ref.state_dict())
    prod = prod.to(dev)
    prod.compute_dtype = torch.float32
    T = 6
    dr, dp = R.Diffusion(ref, timesteps=T), Diffusion(prod, timesteps=T).to(dev)
    g = torch.Generator().manual_seed(11)
    shape = (2, 1, 16, 24)
    cond = torch.randn(2, 1, 16, 24, generator=g)
    x_T = torch.randn(shape, generator=g)
    noise_seq = torch.randn(T, *shape, generator=g)
    y_ref = dr.sample(cond, shape, "cpu", x_T=x_T, noise_seq=noise_seq)
    for use_graph in (False, True):
        y = dp.sample(cond.to(dev), shape, dev, use_graph=use_graph, x_T=x_T, noise_seq=noise_seq.to(dev))
        err = rel(y, y_ref)
        print(f"sampler fp32 vs oracle (graph={use_graph}): rel {err:.3e}")
        assert err < 1e-4
