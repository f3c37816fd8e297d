"""Library reference for the x6 GEMM's MFMA ceiling: the six bf16 products of
an x6 contraction as ONE bf16 GEMM with a 6x longer K (planes concatenated
along K, fp32 output), timed through torch.matmul (hipBLASLt / rocBLAS).
Not a product path -- it tells how close the hand-written k_gemm_x6 runs to
what the vendor GEMM reaches on the same MFMA work.
    python scripts/blas_ref.py"""
import torch

D = torch.device("cuda")
R, K6, U = 405, 25088, 4096
cases = [("fc6_fwd", R, 6 * K6, U), ("fc6_dx", R, 6 * U, K6), ("fc6_dw", K6, 6 * R, U), ("fc7_fwd", R, 6 * U, U)]
g = torch.Generator(device=D).manual_seed(0)


def t(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for lib in ("default", "hipblaslt", "rocblas"):
    try:
        if lib != "default":
            torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:  # noqa: BLE001
        print(lib, "unavailable", e)
        continue
    for name, M, K, N in cases:
        a = torch.randn((M, K), generator=g, device=D).bfloat16()
        b = torch.randn((K, N), generator=g, device=D).bfloat16()
        us = t(lambda: torch.mm(a, b))
        fl = 2.0 * M * K * N
        print(f"{lib:10s} {name:8s} M={M:6d} K={K:6d} N={N:6d} bf16->bf16 {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s "
              f"(x6-equivalent fp32-faithful {fl / 6 / us / 1e6:6.1f})", flush=True)
        try:
            us2 = t(lambda: torch.mm(a, b, out_dtype=torch.float32))
            print(f"{lib:10s} {name:8s} bf16->f32 {us2:8.1f} us  {fl / us2 / 1e6:7.1f} TFLOP/s", flush=True)
        except Exception as e:  # noqa: BLE001
            print("  out_dtype f32 unsupported:", str(e)[:80])
        a32 = a.float()
        b32 = b.float()
        torch.backends.cuda.matmul.allow_tf32 = False
        us3 = t(lambda: torch.mm(a32[:, : K // 6], b32[: K // 6]), iters=10)
        print(f"{lib:10s} {name:8s} fp32 (K/6) {us3:8.1f} us  {2.0 * M * K / 6 * N / us3 / 1e6:7.1f} TFLOP/s",
              flush=True)
        del a, b, a32, b32
