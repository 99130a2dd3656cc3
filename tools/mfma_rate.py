"""MFMA issue rate on the GPU: v_mfma_f32_16x16x16_bf16 vs v_mfma_f32_16x16x32_bf16, 8 independent accumulators per
wave, 256-thread blocks (one wave per SIMD), one block per CU x 4 rounds.  python tools/mfma_rate.py"""
import ctypes
import os

import torch

LIB = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "diag", "libmfma_rate.so"))
LIB.mfma_rate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]


def main():
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    out = torch.zeros(ncu * 4, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    iters = 20000
    for kind, name, flop in ((0, "16x16x16", 2 * 16 * 16 * 16), (1, "16x16x32", 2 * 16 * 16 * 32)):
        LIB.mfma_rate(kind, 100, ctypes.c_void_p(out.data_ptr()), ncu, st)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        LIB.mfma_rate(kind, iters, ctypes.c_void_p(out.data_ptr()), ncu, st)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        n_mfma_per_simd = iters * 8  # one wave per SIMD
        tflops = ncu * 4 * n_mfma_per_simd * 64 * flop / 64 / (ms * 1e-3) / 1e12
        print(f"{name}: {ms:.3f} ms for {iters} x 8 MFMAs per wave -> {ms * 1e-3 / n_mfma_per_simd * 1e9:.2f} ns per MFMA "
              f"per SIMD, {tflops:.0f} TFLOP/s chip-wide", flush=True)


if __name__ == "__main__":
    main()
