"""Bit-exactness of two builds of the halo conv on the same inputs (e.g. an epilogue change): run once per library,
then compare.  usage:
  [CESM_HIP_LIB=lib_a] python tools/epw_check.py dump out_a.pt
  [CESM_HIP_LIB=lib_b] python tools/epw_check.py dump out_b.pt
  python tools/epw_check.py cmp out_a.pt out_b.pt
Shapes: the bench's halo-conv levels with and without bias, residuals, concat inputs and split outputs."""
import sys

import torch

sys.path.insert(0, ".")

SHAPES = [  # (Nb, H, W, C1, C2, Cout, Co1, bias, res)
    (8, 96, 144, 128, 0, 128, 128, True, False),
    (8, 48, 72, 256, 0, 256, 256, False, True),
    (8, 24, 36, 512, 0, 512, 512, True, True),
    (4, 192, 288, 64, 64, 64, 64, True, False),
    (4, 192, 288, 128, 0, 128, 64, False, True),
    (8, 96, 144, 128, 128, 256, 128, True, True),
    (3, 50, 70, 128, 0, 128, 128, True, True),
]


def dump(path):
    from cesm_emulator_amd import kernels as K
    dev = torch.device("cuda")
    out = []
    for idx, (Nb, H, W, C1, C2, Cout, Co1, has_b, has_r) in enumerate(SHAPES):
        g = torch.Generator(device="cpu").manual_seed(idx)
        x1 = torch.randn(Nb, H, W, C1, generator=g).to(dev, torch.bfloat16)
        x2 = torch.randn(Nb, H, W, C2, generator=g).to(dev, torch.bfloat16) if C2 else None
        w = (torch.randn(Cout, C1 + C2, 3, 3, generator=g) * (9 * (C1 + C2)) ** -0.5).to(dev)
        wp = K.conv_pack(w, torch.bfloat16, Cout, C1 + C2, 3, 3, 0, 0)
        b = torch.randn(Cout, generator=g).to(dev) if has_b else None
        r1 = torch.randn(Nb, H, W, Co1, generator=g).to(dev, torch.bfloat16) if has_r else None
        r2 = torch.randn(Nb, H, W, Cout - Co1, generator=g).to(dev, torch.bfloat16) if has_r and Co1 < Cout else None
        y = K.conv_fwd(x1, x2, wp, b, (H, W, Cout, 3, 3, 1, 1, 1), res=r1, res2=r2,
                       out_split=Co1 if Co1 < Cout else None)
        ys = y if isinstance(y, tuple) else (y,)
        out.append([t.cpu() for t in ys])
        print(idx, K.lib().cesm_conv_fwd_variant(1, Nb, H, W, C1, C2, H, W, Cout, Co1, 3, 3, 1, 1, 1).decode(),
              flush=True)
    torch.save(out, path)


def cmp(a, b):
    A, B = torch.load(a), torch.load(b)
    bad = 0
    for idx, (ya, yb) in enumerate(zip(A, B)):
        for ta, tb in zip(ya, yb):
            eq = torch.equal(ta.view(torch.int16), tb.view(torch.int16))
            nd = int((ta.view(torch.int16) != tb.view(torch.int16)).sum())
            print(idx, SHAPES[idx], "bit-identical" if eq else f"DIFFER in {nd} of {ta.numel()}")
            bad += 0 if eq else 1
    print("all bit-identical" if bad == 0 else f"{bad} outputs differ")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
