"""Library GEMM reference points for the mat-mat shapes (calibration of the int8 / f16 MFMA
floors on this part, no block scales): torch._int_mm (int8 x int8 -> int32, hipBLASLt) and
torch.matmul in f16, M x K times K x N, mean of back-to-back launches by HIP events."""
import sys
import torch

torch.cuda.set_device(0)
for sh in sys.argv[1:] or ["512:4096:4096", "2048:4096:4096", "512:4096:11008"]:
    M, K, N = map(int, sh.split(":"))
    a8 = torch.randint(-127, 127, (M, K), dtype=torch.int8, device="cuda")
    b8 = torch.randint(-127, 127, (N, K), dtype=torch.int8, device="cuda").t()
    a16 = torch.randn(M, K, dtype=torch.float16, device="cuda")
    b16 = torch.randn(N, K, dtype=torch.float16, device="cuda").t()
    for name, fn in (("int8 _int_mm", lambda: torch._int_mm(a8, b8)), ("f16 matmul", lambda: a16 @ b16)):
        try:
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            print(f"{name:14s} M={M} K={K} N={N}: {us:8.2f} us  {2 * M * K * N / us / 1e6:8.1f} T(FL)OP/s", flush=True)
        except Exception as ex:  # noqa: BLE001
            print(f"{name} {sh}: {ex}")
