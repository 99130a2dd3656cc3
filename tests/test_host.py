"""CPU tests of the host-side logic: C-ABI exports, config surface, data sampling/gather semantics
vs the dataset restatement, sharding vs DistributedSampler, FLOP accounting."""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ C ABI
def test_library_exports_every_header_symbol():
    from cesm_emulator_amd import _lib
    from cesm_emulator_amd.build import build
    build()
    decls = _lib.parse_header()
    assert len(decls) >= 30
    handle = ctypes.CDLL(str(_lib.LIBPATH))
    missing = [n for n in decls if not hasattr(handle, n)]
    assert not missing, missing
    # and nothing exported that the header does not declare
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIBPATH)], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T cesm_" in l}
    assert exported == set(decls), exported ^ set(decls)
    _lib.lib()  # argtypes bind cleanly


def test_kernels_refuse_cpu_tensors():
    from cesm_emulator_amd import kernels as K
    with pytest.raises(RuntimeError):
        K.ln_fwd(torch.zeros(4, 64), torch.ones(64))


def test_model_refuses_cpu_inputs():
    from cesm_emulator_amd.model import UNet
    u = UNet()
    with pytest.raises(RuntimeError, match="GPU"):
        u(torch.zeros(1, 1, 8, 8), torch.zeros(1, 1, 8, 8), torch.tensor([1]))
    with pytest.raises(ValueError):
        u(torch.zeros(1, 1, 8), torch.zeros(1, 1, 8, 8), torch.tensor([1]))
    with pytest.raises(ValueError, match="Frame mismatch"):
        u(torch.zeros(1, 1, 2, 8, 8), torch.zeros(1, 1, 3, 8, 8), torch.tensor([1]))


# ------------------------------------------------------------------ config
def test_configs_load_and_override():
    from cesm_emulator_amd.config import load_config, apply_overrides, dataset_kwargs
    for name in ("baseline", "more_blocks"):
        cfg = load_config(os.path.join(ROOT, "config", name))
        apply_overrides(cfg, ["dataset.K=12", "dataset.crop_hw=0", "train.batch_size=5", "train.lr=0.001",
                              "train.use_amp=false", "new.key=abc"])
        assert cfg["dataset"]["K"] == 12 and cfg["train"]["batch_size"] == 5
        assert cfg["train"]["lr"] == 0.001 and cfg["train"]["use_amp"] is False and cfg["new"]["key"] == "abc"
        assert dataset_kwargs(cfg)["crop_hw"] is None
    with pytest.raises(ValueError):
        apply_overrides({}, ["novalue"])


def test_build_model_from_config_matches_reference_kwargs():
    from cesm_emulator_amd.config import load_config
    from cesm_emulator_amd.train import build_model_from_config
    from oracle import ref_cpu as R
    for name in ("baseline", "more_blocks"):
        cfg = load_config(os.path.join(ROOT, "config", name))
        a = build_model_from_config(cfg["unet"])
        b = R.UNet(**R.config_unet_kwargs(cfg["unet"]))
        assert list(a.state_dict()) == list(b.state_dict())


# ------------------------------------------------------------------ data
@pytest.mark.parametrize("center,crop,p", [(True, (7, 9), 0.5), (True, None, 0.5), (False, (5, 5), 1.0),
                                           (True, (10, 12), 0.0)])
def test_sampler_and_host_gather_match_dataset(center, crop, p):
    from cesm_emulator_amd.data import WindowSampler, host_gather
    from oracle.ref_data import WindowedAllMembersDatasetRef
    rng = np.random.default_rng(0)
    T, M, H, W, K = 11, 4, 10, 12, 5
    cond = rng.standard_normal((T, M, 1, H, W)).astype(np.float32)
    tgt = rng.standard_normal((T, M, 1, H, W)).astype(np.float32)
    ref = WindowedAllMembersDatasetRef(cond, tgt, K=K, center=center, crop_hw=crop, time_reverse_p=p)
    smp = WindowSampler(T, M, H, W, K, center, crop, "random", p)
    assert len(ref) == len(smp)
    idx = list(range(len(ref)))[::3]
    np.random.seed(42)
    exp = [ref[i] for i in idx]
    np.random.seed(42)
    items = smp.items(idx)
    h, w = smp.hw
    oc = np.zeros((len(idx), 1, K, h, w), np.float32)
    ox = np.zeros((len(idx), 1, h, w), np.float32)
    host_gather(cond[:, :, 0], tgt[:, :, 0], items, K, h, w, center, oc, ox)
    for n, (c, x) in enumerate(exp):
        np.testing.assert_array_equal(oc[n], c.numpy())
        np.testing.assert_array_equal(ox[n], x.numpy())


def test_shard_indices_matches_distributed_sampler():
    from torch.utils.data.distributed import DistributedSampler
    from cesm_emulator_amd.data import shard_indices
    n = 23
    for world in (1, 2, 3):
        for rank in range(world):
            for epoch in (0, 3):
                s = DistributedSampler(list(range(n)), num_replicas=world, rank=rank, shuffle=True, seed=0)
                s.set_epoch(epoch)
                exp = list(iter(s))
                got = [i for b in shard_indices(n, 4, rank, world, True, 0, epoch) for i in b]
                assert got == exp


def test_zscore_matches_train_py():
    from cesm_emulator_amd.data import zscore
    a = np.random.default_rng(1).standard_normal((3, 2, 4, 5)).astype(np.float32) * 7 + 3
    z, m, s = zscore(a)
    np.testing.assert_allclose(z, (a - a.mean()) / (a.std() + 1e-8), rtol=1e-6)


# ------------------------------------------------------------------ accounting
def test_flop_count_reconciles_with_survey():
    from cesm_emulator_amd.flops import unet_forward_macs
    from oracle import ref_cpu as R
    net = R.UNet(ch_mults=(1, 2, 4, 8)).net
    per_voxel = unet_forward_macs(net, 12, 192, 288) / (12 * 192 * 288)
    # 1,816,256 + 1,880*F MAC/voxel, plus the out_conv.0 block2 + res_conv that
    # SURVEY omitted (64*64*9 + 128*64 = 45,056 MAC/voxel) and the tiny time-MLP linears
    survey = 1_816_256 + 1_880 * 12
    assert abs(per_voxel - (survey + 45_056)) < 5


# ------------------------------------------------------------------ kernel dispatch (host-only queries)
def test_gn_epilogue_slot_counts():
    """GroupNorm partial slots the Block convs write from their epilogue (cesm_conv_gn_nslot, host only):
    the warp-specialized conv per (frame, 8x32 tile, 64-pixel quarter), the halo conv per (frame, tile, wave = 64-pixel
    quarter); 0 where the kernel has no partials (fp32 generic conv, 1x1, B not dividing the batch) -> the separate
    statistics pass"""
    from cesm_emulator_amd import kernels as K
    bf = torch.bfloat16
    g3 = lambda H, W, C: (H, W, C, 3, 3, 1, 1, 1)  # noqa: E731
    x = torch.empty(96, 192, 288, 64, dtype=bf)
    assert K.conv_gn_nslot(x, None, g3(192, 288, 64), 8) == 12 * (24 * 9) * 4
    assert K.conv_gn_nslot(x, x, g3(192, 288, 64), 8) == 12 * (16 * 8) * 4  # 12 x 36 tiles (448-px blocks)
    x1 = torch.empty(96, 96, 144, 128, dtype=bf)
    assert K.conv_gn_nslot(x1, None, g3(96, 144, 128), 8) == 12 * (8 * 4) * 4
    assert K.conv_gn_nslot(x1, None, g3(96, 144, 128), 7) == 0
    assert K.conv_gn_nslot(x1.float(), None, g3(96, 144, 128), 8) == 0
    assert K.conv_gn_nslot(x1, None, (96, 144, 128, 1, 1, 1, 0, 1), 8) == 0


def test_bench_shape_dispatch_table():
    """which kernel each bench-shape conv reaches (more_blocks 192x288, B*F = 96; cesm_conv_*_variant
    runs the launchers' own selection on the host).  tests/test_gpu_prod_parity.py covers these."""
    from cesm_emulator_amd import kernels as K
    bf = torch.bfloat16
    N = 96
    fv = lambda *a: K.conv_fwd_variant(bf, N, *a)  # noqa: E731
    wv = lambda *a, **k: K.conv_wgrad_variant(bf, N, *a, **k)  # noqa: E731
    # level 0, 64 -> 64 3x3 (fwd and dgrad): the warp-specialized persistent conv
    assert fv(192, 288, 64, 0, 192, 288, 64, 64, 3, 3, 1, 1, 1) == "conv3x3ws_kernel<32>"
    assert wv(192, 288, 64, 0, 192, 288, 64, 64, 3, 3, 1, 1, 1) == "wgrad3x3c64_kernel"
    # level-0 concat inputs (up path / out_conv: 64 + 64 -> 64)
    assert fv(192, 288, 64, 64, 192, 288, 64, 64, 3, 3, 1, 1, 1) == "conv3x3_bf16_kernel<36>"
    # levels 1-3 (144, 72, 36 wide)
    assert fv(96, 144, 128, 0, 96, 144, 128, 128, 3, 3, 1, 1, 1) == "conv3x3_bf16_kernel<36>"
    assert fv(48, 72, 256, 0, 48, 72, 256, 256, 3, 3, 1, 1, 1) == "conv3x3_bf16_kernel<36>"
    assert fv(24, 36, 512, 0, 24, 36, 512, 512, 3, 3, 1, 1, 1) == "conv3x3_bf16_kernel<36>"
    assert wv(24, 36, 512, 0, 24, 36, 512, 512, 3, 3, 1, 1, 1) == "wgrad3x3w36c64_kernel"
    # 768-channel qkv weight gradient of the fused attention blocks; the SLA to_out with its bias
    assert wv(192, 288, 64, 0, 192, 288, 768, 768, 1, 1, 1, 0, 1) == "wgrad_wide_kernel<256,false>"
    # ... at C = 128 / 256 / 512: square 256 x BN tiles (dY read once per row tile, round 6)
    assert wv(96, 144, 128, 0, 96, 144, 768, 768, 1, 1, 1, 0, 1) == "wgrad_sq_kernel<256,128>"
    assert wv(48, 72, 256, 0, 48, 72, 768, 768, 1, 1, 1, 0, 1) == "wgrad_sq_kernel<256,256>"
    assert wv(24, 36, 512, 0, 24, 36, 768, 768, 1, 1, 1, 0, 1) == "wgrad_sq_kernel<256,256>"
    assert wv(24, 36, 512, 0, 24, 36, 768, 768, 1, 1, 1, 0, 1, with_bias=True) == "wgrad_sq_kernel<256,256,true>"
    # the level-0 temporal to_out (256 -> 64, no bias): 64 x 256 tiles
    assert wv(192, 288, 256, 0, 192, 288, 64, 64, 1, 1, 1, 0, 1) == "wgrad_sq_kernel<64,256>"
    assert wv(192, 288, 256, 0, 192, 288, 64, 64, 1, 1, 1, 0, 1, with_bias=True) == "wgrad_sq_kernel<64,256,true>"
    # 1x1 res_conv / to_qkv GEMMs, down- and up-sampling
    assert fv(192, 288, 64, 0, 192, 288, 768, 768, 1, 1, 1, 0, 1) == "gemm1x1_kernel<128>"
    # down / up (4x4 stride 2 and its transpose; tile width chosen on the low-resolution grid)
    assert fv(192, 288, 64, 0, 96, 144, 64, 64, 4, 4, 2, 1, 1) == "convs2_bf16_kernel<32,down>"
    assert fv(96, 144, 64, 0, 192, 288, 64, 64, 4, 4, 1, 2, 2) == "convs2_bf16_kernel<32,up>"
    assert fv(96, 144, 128, 0, 48, 72, 128, 128, 4, 4, 2, 1, 1) == "convs2_bf16_kernel<36,down>"
    assert fv(24, 36, 256, 0, 48, 72, 256, 256, 4, 4, 1, 2, 2) == "convs2_bf16_kernel<36,up>"
    assert wv(192, 288, 64, 0, 96, 144, 64, 64, 4, 4, 2, 1, 1) == "wgrads2_bf16_kernel"
    assert wv(192, 288, 64, 0, 96, 144, 64, 64, 4, 4, 2, 1, 1, with_bias=True) == "wgrad_wide_kernel<64,true>"
    assert wv(48, 72, 256, 0, 24, 36, 256, 256, 4, 4, 2, 1, 1) == "wgrad_wide_kernel<256,false>"
    # fp32 parity mode: the generic kernels
    assert K.conv_fwd_variant(torch.float32, N, 192, 288, 64, 0, 192, 288, 64, 64, 3, 3, 1, 1, 1) == \
        "conv_fwd_kernel<float,64>"
    # arguments cesm_conv_fwd rejects
    assert K.conv_fwd_variant(bf, N, 8, 8, 48, 0, 8, 8, 64, 64, 3, 3, 1, 1, 1) == "invalid"


def test_tflash_dq_dispatch():
    """the temporal attention core backward (cesm_tflash_bwd_variant, host only): the one-pass fused kernel for every
    F >= 8 (round 5), the two-kernel form (block-per-pixel dq kernel + the dk / dv kernel) below"""
    from cesm_emulator_amd import kernels as K
    assert K.tflash_bwd_variant(120, 192 * 288) == "tflash_bwd_fused_kernel<8>"
    assert K.tflash_bwd_variant(120, 48 * 72) == "tflash_bwd_fused_kernel<8>"
    assert K.tflash_bwd_variant(17, 40) == "tflash_bwd_fused_kernel<2>"
    assert K.tflash_bwd_variant(12, 192 * 288) == "tflash_bwd_fused_kernel<1>"
    assert K.tflash_bwd_variant(7, 192 * 288) == "tflash_bwd_q_kernel<1>"
    assert K.tflash_bwd_variant(40, 200 * 200) == "tflash_bwd_fused_kernel<3>"
    assert K.tflash_bwd_variant(1, 64) == "tflash_bwd_q_kernel<1>"
    assert K.tflash_bwd_variant(129, 64) == "invalid"


def test_bench_probe_wrappers_accept_kernel_signatures():
    """bench.py's live kernel probe replaces kernels.* functions with wrappers that compute a label and the work of
    the call: every wrapper must accept every parameter of the function it wraps (a new keyword on a kernels.*
    function would otherwise raise inside the timed bench step)"""
    import ast
    import inspect
    import os
    from cesm_emulator_amd import kernels as K
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")).read()
    probe = [n for n in ast.parse(src).body if isinstance(n, ast.ClassDef) and n.name == "KernelProbe"][0]
    init = [n for n in probe.body if isinstance(n, ast.FunctionDef) and n.name == "__init__"][0]
    checked = 0
    for n in init.body:
        if isinstance(n, ast.FunctionDef) and hasattr(K, n.name):
            have = [a.arg for a in n.args.args]
            want = list(inspect.signature(getattr(K, n.name)).parameters)
            assert [p for p in want if p not in have] == [], n.name
            checked += 1
    assert checked >= 15
