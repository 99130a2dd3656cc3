"""Warp-specialized 3x3 conv (conv3x3ws_kernel) against the kernels it replaces: every bench-step 3x3 shape, plain /
residual / GroupNorm-partial launches, outputs compared bit for bit (same MFMA order per output) and timed.

  python tools/ws_check.py            (spawns itself twice: CESM_NO_CONV_WS=1 and CESM_CONV_WS=1, then compares)
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (Nb, H, W, C1, C2, Cout): the bench step's 3x3 stride-1 shapes (B = 8, F = 12 -> Nb = 96)
SHAPES = [
    (96, 192, 288, 64, 0, 64),     # level 0 (conv3x3p today)
    (96, 192, 288, 64, 64, 64),    # level-0 concat (decoder)
    (96, 96, 144, 128, 0, 128),    # level 1
    (96, 96, 144, 128, 128, 128),  # level-1 concat
    (96, 48, 72, 256, 0, 256),     # level 2
    (96, 24, 36, 512, 0, 512),     # level 3 (stays on the halo conv: 84 % tile cover)
    (6, 20, 96, 64, 0, 64),        # small / partial tiles
    (4, 30, 72, 128, 64, 128),
]


def run(out_path):
    import torch
    from cesm_emulator_amd import kernels as K
    dev = torch.device("cuda")
    res = {}
    bf = torch.bfloat16
    for (Nb, H, W, C1, C2, Co) in SHAPES:
        g = torch.Generator(device=dev).manual_seed(Nb * 7 + H + W + C1 + C2)
        x1 = torch.randn(Nb, H, W, C1, device=dev, generator=g).to(bf)
        x2 = torch.randn(Nb, H, W, C2, device=dev, generator=g).to(bf) if C2 else None
        w = torch.randn(Co, C1 + C2, 3, 3, device=dev, generator=g) * (9 * (C1 + C2)) ** -0.5
        wp = K.conv_pack(w, bf, Co, C1 + C2, 3, 3, False, False)
        b = torch.randn(Co, device=dev, generator=g)
        r = torch.randn(Nb, H, W, Co, device=dev, generator=g).to(bf)
        geom = (H, W, Co, 3, 3, 1, 1, 1)
        var = K.conv_fwd_variant(bf, Nb, H, W, C1, C2, H, W, Co, Co, 3, 3, 1, 1, 1)
        y = K.conv_fwd(x1, x2, wp, b, geom)
        yr = K.conv_fwd(x1, x2, wp, b, geom, res=r)
        B = 8 if Nb % 8 == 0 else 2
        nslot = K.conv_gn_nslot(x1, x2, geom, B)
        gn = None
        if nslot > 0:
            yg, part = K.conv_fwd_gn(x1, x2, wp, b, geom, B, nslot)
            gn = (yg.cpu(), K.gn_stats_part(part, Nb // B * H * W, 8).cpu())
        torch.cuda.synchronize()
        reps = 5 if Nb >= 96 else 20
        t0 = time.perf_counter()
        for _ in range(reps):
            K.conv_fwd(x1, x2, wp, b, geom)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps * 1e6
        res[(Nb, H, W, C1, C2, Co)] = dict(var=var, y=y.cpu(), yr=yr.cpu(), gn=gn, us=dt)
        print(f"  {os.environ.get('CESM_CONV_WS', '0')} {Nb}x{H}x{W} {C1}+{C2}->{Co}: {var:32s} {dt:8.1f} us", flush=True)
    torch.save(res, out_path)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--run":
        run(sys.argv[2])
        return
    outs = {}
    for ws in ("0", "1"):
        path = f"/tmp/ws_check_{ws}.pt"
        env = dict(os.environ, CESM_CONV_WS=ws, CESM_NO_CONV_WS="1" if ws == "0" else "0")
        r = subprocess.run([sys.executable, __file__, "--run", path], env=env, timeout=600)
        if r.returncode != 0:
            sys.exit(f"run CESM_CONV_WS={ws} failed: {r.returncode}")
        import torch
        outs[ws] = torch.load(path, weights_only=False)
    ok = True
    for k in outs["0"]:
        a, b = outs["0"][k], outs["1"][k]
        eq_y = bool((a["y"] == b["y"]).all())
        # residual: conv3x3p and the warp-specialized kernel round (acc + bias) to bf16 before adding it, the halo conv
        # adds in fp32 -> at most one bf16 rounding step apart
        eq_r = bool((a["yr"] == b["yr"]).all())
        if not eq_r:  # one extra bf16 rounding of (acc + bias) at |y| plus the final rounding at |out|
            ra, rb, ya = a["yr"].float(), b["yr"].float(), a["y"].float()
            tol = (ya.abs() + ra.abs()) * 2.0 ** -8 * 1.01 + 1e-6
            eq_r = bool(((ra - rb).abs() <= tol).all())
        dy = (a["y"].float() - b["y"].float()).abs().max().item()
        gnmsg = ""
        if a["gn"] is not None and b["gn"] is not None:
            eq_g = bool((a["gn"][0] == b["gn"][0]).all())
            dst = (a["gn"][1] - b["gn"][1]).abs().max().item()
            gnmsg = f" gn_y {'==' if eq_g else '!='} stats maxdiff {dst:.2e}"
            ok = ok and eq_g and dst < 1e-4
        ok = ok and eq_y and eq_r
        print(f"{k}: {a['var']} {a['us']:.1f} us -> {b['var']} {b['us']:.1f} us ({a['us'] / b['us']:.2f}x); "
              f"y {'==' if eq_y else '!='} (maxdiff {dy:.2e}) yres {'==' if eq_r else '!='}{gnmsg}")
    print("WS CHECK", "PASS" if ok else "FAIL")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
