"""Reference-format checkpoints: files in the layout train.py:1154-1165
writes load into cesm_emulator_amd (train.py:915-946 / inference.py:47-73 semantics) and vice versa.

CPU: model weights + diffusion buffers + epoch/config round trips between the oracle (the reference's
module tree) and the drop-in UNet/Diffusion, both directions, strict key equality.
GPU: FusedAdamW.state_dict() is a torch.optim.AdamW state dict (loads into AdamW over the reference's
parameter list, frozen rotary freqs included) and AdamW's state dict loads back into FusedAdamW.
"""
import io

import pytest
import torch

from cesm_emulator_amd import checkpoint as CK
from cesm_emulator_amd.model import UNet, Diffusion
from oracle import ref_cpu as R

CFG = {"unet": {"in_channels": 2, "out_channels": 1, "base_ch": 64, "ch_mults": [1, 2, 4], "groups": 8},
       "train": {"timesteps": 1000, "beta_schedule": "linear"}}


def _ref_trained(tmp_path):
    torch.manual_seed(3)
    ref = R.Diffusion(R.UNet(ch_mults=(1, 2, 4)))
    opt = R.make_optimizer(ref)
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(1, 1, 16, 24, generator=g)
    cond = torch.randn(1, 1, 2, 16, 24, generator=g)
    R.train_step(ref, opt, x0, cond, t=torch.tensor([5]), noise=torch.randn(1, 1, 16, 24, generator=g))
    path = tmp_path / "ckpt_epoch_0007.pt"
    CK.save_checkpoint(path, ref, opt, 7, CFG)  # same dict as train.py:1159-1165
    return ref, opt, path


def test_reference_checkpoint_loads_into_dropin(tmp_path):
    ref, _, path = _ref_trained(tmp_path)
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"epoch", "model", "diffusion_buffers", "optimizer", "config"}
    assert all(not k.startswith("model.") for k in ck["model"])
    assert set(ck["diffusion_buffers"]) == {"betas", "alphas", "alphas_cumprod", "alphas_cumprod_prev",
                                            "sqrt_alphas_cumprod", "sqrt_one_minus_alphas_cumprod",
                                            "sqrt_recip_alphas", "posterior_variance"}
    torch.manual_seed(99)  # different init: everything must come from the file
    unet = UNet(ch_mults=(1, 2, 4))
    diff = Diffusion(unet)
    assert CK.load_checkpoint(path, unet, diff, None, device="cpu") == 8
    for (k, a), (k2, b) in zip(ref.state_dict().items(), diff.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k
    d2, cfg = CK.load_diffusion_from_checkpoint(path, device="cpu")
    assert cfg == CFG and not d2.training and not any(p.requires_grad for p in d2.parameters())
    for (k, a), (_, b) in zip(ref.state_dict().items(), d2.state_dict().items()):
        assert torch.equal(a, b), k


def test_dropin_checkpoint_loads_into_reference(tmp_path):
    torch.manual_seed(5)
    diff = Diffusion(UNet(ch_mults=(1, 2, 4, 8)))
    path = tmp_path / "ours.pt"
    CK.save_checkpoint(path, diff, None, 2, CFG)
    ck = torch.load(path, weights_only=True)
    torch.manual_seed(6)
    ref = R.Diffusion(R.UNet(ch_mults=(1, 2, 4, 8)))
    ref.model.load_state_dict(ck["model"], strict=True)
    st = ref.state_dict()
    st.update(ck["diffusion_buffers"])
    ref.load_state_dict(st, strict=True)
    for (k, a), (_, b) in zip(diff.state_dict().items(), ref.state_dict().items()):
        assert torch.equal(a, b), k


@pytest.mark.gpu
def test_fused_adamw_state_is_torch_adamw_layout(dev):
    from cesm_emulator_amd.optim import FusedAdamW
    from cesm_emulator_amd.train import train_step
    torch.manual_seed(3)
    ref = R.Diffusion(R.UNet(ch_mults=(1, 2, 4)))
    torch.manual_seed(3)
    net = UNet(ch_mults=(1, 2, 4))
    net.load_state_dict(ref.model.state_dict())
    net = net.to(dev)
    net.compute_dtype = torch.float32
    diff = Diffusion(net).to(dev)
    opt = FusedAdamW(diff.parameters(), lr=2e-4, weight_decay=1e-4, max_grad_norm=1.0)
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(2, 1, 16, 24, generator=g).to(dev)
    cond = torch.randn(2, 1, 2, 16, 24, generator=g).to(dev)
    for _ in range(2):
        train_step(diff, opt, x0, cond, 1.0, t=torch.tensor([3, 600], device=dev), noise=torch.randn_like(x0))
    buf = io.BytesIO()
    torch.save(opt.state_dict(), buf)
    buf.seek(0)
    sd = torch.load(buf, weights_only=True)
    # the reference's optimizer (train.py:1077-1083) over the reference's parameter list accepts it
    ref_opt = R.make_optimizer(ref)
    ref_opt.load_state_dict(sd)
    names = [n for n, _ in ref.named_parameters()]
    ours = dict(diff.named_parameters())
    off = {id(q): o for q, o in zip(opt.flat.params, opt.flat.offsets)}
    assert len(ref_opt.state) == sum(p.requires_grad for p in ref.parameters())
    for i, p in enumerate(ref.parameters()):
        if not p.requires_grad:
            assert p not in ref_opt.state  # frozen rotary freqs: no state, as in torch
            continue
        st = ref_opt.state[p]
        assert int(st["step"]) == 2
        a = opt.exp_avg[off[id(ours[names[i]])]:][:p.numel()]
        assert torch.equal(st["exp_avg"].reshape(-1), a.cpu()), names[i]
    # and AdamW's own state dict loads back into FusedAdamW
    opt2 = FusedAdamW(Diffusion(UNet(ch_mults=(1, 2, 4)).to(dev)).to(dev).parameters())
    opt2.load_state_dict(ref_opt.state_dict())
    assert opt2.step_count == 2
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq)
    assert opt2.param_groups[0]["lr"] == 2e-4 and tuple(opt2.param_groups[0]["betas"]) == (0.9, 0.999)
