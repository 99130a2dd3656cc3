"""Per-wave dq kernel (tflash_bwd_qw_kernel) against the round-3 block-per-pixel dq kernels (CESM_TF_NO_QW=1):
temporal-attention backward at the F = 120 level shapes and F = 12 / 24 / 40 windows, dqkv / rel-pos table
gradient compared and timed.

  python tools/tf_qw_check.py            (spawns itself twice: CESM_TF_NO_QW=1 and CESM_TF_QW=1, then compares)
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (F, H, W, B)
SHAPES = [(120, 192, 288, 1), (120, 96, 144, 1), (120, 48, 72, 1), (120, 24, 36, 1), (24, 48, 72, 4),
          (40, 24, 36, 2), (17, 10, 12, 3), (12, 24, 36, 8)]


def run(out_path):
    import torch
    from cesm_emulator_amd import kernels as K
    dev = torch.device("cuda")
    res = {}
    for (F, H, W, B) in SHAPES:
        HW = H * W
        g = torch.Generator(device=dev).manual_seed(F * 131 + H + W + B)
        qkv = torch.randn(B * F * HW, 768, device=dev, generator=g).to(torch.bfloat16)
        bias = K.relpos_fwd(torch.randn(32, 8, device=dev, generator=g), F)
        rot = K.rope_table(1.0 / (10000 ** (torch.arange(0, 32, 2, device=dev).float() / 32)), F)
        out, lse = K.tattn_fwd(qkv, bias, rot, B, F, HW, 32 ** -0.5)
        dout = torch.randn(out.shape, device=dev, generator=g).to(out.dtype)
        dtable = torch.zeros(32, 8, device=dev)
        dqkv = K.tattn_bwd(qkv, out, dout, lse, bias, rot, dtable, B, F, HW, 32 ** -0.5)
        torch.cuda.synchronize()
        reps = 3 if HW * F * B > 10 ** 6 else 10
        t0 = time.perf_counter()
        for _ in range(reps):
            K.tattn_bwd(qkv, out, dout, lse, bias, rot, torch.zeros(32, 8, device=dev), B, F, HW, 32 ** -0.5)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps * 1e6
        # dq columns (0..255) of a bounded sample of rows (the full tensor at 192x288 is 10 GB)
        n = dqkv.shape[0]
        idx = torch.arange(0, n, max(1, n // 65536), device=dev)
        res[(F, H, W, B)] = dict(dq=dqkv[idx].cpu(), dt=dtable.cpu(), us=dt)
        print(f"  {os.environ.get('CESM_TF_NO_QW', '0')} F={F} {H}x{W} B={B}: bwd {dt:9.1f} us", flush=True)
        del qkv, out, dout, dqkv
        torch.cuda.empty_cache()
    torch.save(res, out_path)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--run":
        run(sys.argv[2])
        return
    outs = {}
    for v in ("1", "0"):
        path = f"/tmp/tf_qw_{v}.pt"
        env = dict(os.environ, CESM_TF_NO_QW=v, CESM_TF_QW="0" if v == "1" else "1")
        r = subprocess.run([sys.executable, "-u", __file__, "--run", path], env=env, timeout=900)
        if r.returncode != 0:
            sys.exit(f"run CESM_TF_NO_QW={v} failed: {r.returncode}")
        import torch
        outs[v] = torch.load(path, weights_only=True)
    ok = True
    for k in outs["1"]:
        a, b = outs["1"][k], outs["0"][k]
        dqa, dqb = a["dq"].float(), b["dq"].float()
        # q-gradient columns; the round-3 kernel at >= 8192 pixels takes D = sum P dP instead of dO . O
        cols = slice(0, 256)
        scale = dqa[:, cols].abs().max().item() + 1e-12
        e_dq = (dqa[:, cols] - dqb[:, cols]).abs().max().item() / scale
        kv_eq = bool(torch.equal(a["dq"][:, 256:], b["dq"][:, 256:]))
        e_dt = ((a["dt"] - b["dt"]).abs().max() / (a["dt"].abs().max() + 1e-12)).item()
        good = e_dq < 2e-2 and e_dt < 2e-3
        ok = ok and good
        print(f"{k}: old {a['us']:.1f} us -> qw {b['us']:.1f} us ({a['us'] / b['us']:.2f}x); dq rel {e_dq:.2e} "
              f"dkv {'==' if kv_eq else '!='} dtable rel {e_dt:.2e} {'ok' if good else 'BAD'}")
    print("TF QW CHECK", "PASS" if ok else "FAIL")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
