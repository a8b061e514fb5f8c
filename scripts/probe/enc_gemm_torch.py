"""Reference point for the encoder GEMMs: the library
GEMM (torch.nn.functional.linear -> hipBLASLt on ROCm) on the shapes of one
32-clip large-v3 batch, bf16 operands, f32 accumulation, no epilogue. Prints
TFLOP/s and the fraction of the dense bf16 peak (2.5 PFLOP/s) per shape, to
compare with gemm_big's per-launch times in the kernel trace (which include
the fused epilogues). Not part of the product or its tests.

    python scripts/probe/enc_gemm_torch.py
"""
import json

import torch

M = 32 * 1500  # rows: 32 clips x 1500 encoder frames
SHAPES = {  # name: (N, K), W stored [N][K] as in ggml
    "qkv": (3 * 1280, 1280),
    "out": (1280, 1280),
    "ffn1": (5120, 1280),
    "ffn2": (1280, 5120),
    "cross_kv_all_layers": (2 * 32 * 1280, 1280),
}
PEAK = 2500.0


def main():
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    res = {}
    for name, (n, k) in SHAPES.items():
        a = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.nn.functional.linear(a, w)
        torch.cuda.synchronize()
        reps = 10 if n * k < 50_000_000 else 3
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            torch.nn.functional.linear(a, w)
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) * 1e3 / reps
        tf = 2.0 * M * n * k / us / 1e6
        res[name] = {"M": M, "N": n, "K": k, "us": round(us, 1), "tflops": round(tf, 1),
                     "frac": round(tf / PEAK, 3)}
        print(json.dumps({name: res[name]}), flush=True)
        del a, w
        torch.cuda.empty_cache()
    print(json.dumps({"library_gemm_bf16": res}), flush=True)


if __name__ == "__main__":
    main()
