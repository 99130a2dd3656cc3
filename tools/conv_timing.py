"""Time every conv launch (fwd/dgrad and wgrad) of one bench training step with HIP events and print
per-shape totals, TFLOP/s and share: python tools/conv_timing.py [bench args...]"""
import collections
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from cesm_emulator_amd import kernels as K  # noqa: E402
import bench  # noqa: E402

REC = []
ACTIVE = [False]


def wrap(name, fn, flop_of):
    def w(*a, **k):
        if not ACTIVE[0]:
            return fn(*a, **k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn(*a, **k)
        e.record()
        REC.append((name, flop_of(*a, **k), s, e))
        return r
    return w


def key_fwd(x1, x2, wp, bias, geom, **k):
    Ho, Wo, Cout, KH, KW, St, Pd, U = geom
    cin = x1.shape[3] + (0 if x2 is None else x2.shape[3])
    taps = KH * KW if U == 1 else KH * KW // (U * U)
    d = f"N{x1.shape[0]} {x1.shape[1]}x{x1.shape[2]}x{cin} -> {Ho}x{Wo}x{Cout} k{KH} s{St} u{U}"
    return d, 2.0 * x1.shape[0] * Ho * Wo * Cout * cin * taps


def key_wg(x1, x2, dy1, dy2, dw, geom, swap, flip, accumulate=True, **k):
    Ho, Wo, Cout, KH, KW, St, Pd, U = geom
    cin = x1.shape[3] + (0 if x2 is None else x2.shape[3])
    taps = KH * KW if U == 1 else KH * KW // (U * U)
    d = f"N{x1.shape[0]} {x1.shape[1]}x{x1.shape[2]}x{cin} -> {Ho}x{Wo}x{Cout} k{KH} s{St} u{U}"
    return d, 2.0 * x1.shape[0] * Ho * Wo * Cout * cin * taps


def key_fwd_gn(x1, x2, wp, bias, geom, B, nslot, **k):
    return key_fwd(x1, x2, wp, bias, geom)


def main():
    K.conv_fwd = wrap("fwd", K.conv_fwd, key_fwd)
    K.conv_fwd_gn = wrap("fwdgn", K.conv_fwd_gn, key_fwd_gn)
    K.conv_wgrad = wrap("wgrad", K.conv_wgrad, key_wg)
    sys.argv = ["bench.py", "--steps", "1", "--warmup", "2", "--no-cpu-baseline", "--other-configs", ""] + sys.argv[1:]
    import cesm_emulator_amd.train as T
    ts = T.train_step
    calls = [0]

    def step(*a, **k):
        calls[0] += 1
        ACTIVE[0] = calls[0] == 3  # the timed step
        return ts(*a, **k)
    T.train_step = step  # bench.main() imports train_step from the module at call time
    bench.main()
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    tot = 0.0
    for name, (d, flop), s, e in REC:
        ms = s.elapsed_time(e)
        a = agg[(name, d)]
        a[0] += 1
        a[1] += ms
        a[2] += flop
        tot += ms
    print(f"conv total {tot:.2f} ms in the step")
    for (name, d), (n, ms, flop) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{ms:7.3f} ms {n:3d}x {flop / ms / 1e9:7.1f} TF/s  {name:5s} {d}")


if __name__ == "__main__":
    main()
