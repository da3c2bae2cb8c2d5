"""Library FP64 GEMM timings (torch.mm -> hipBLASLt / rocBLAS) at the chi2 T GEMM and Gram shapes of the
TrackSIM workloads, for comparison with k_gemm_HPg_tiled / k_gram_mfma (rocprof per-launch times)."""
import torch

dev = "cuda"
for name, m, n in [("cfg5", 74568, 242), ("cfg4", 80691, 172), ("cfg3t", 30184, 154)]:
    H = torch.randn(m, 256, dtype=torch.float64, device=dev)[:, :n]  # ld 256 like H_all
    P = torch.randn(n, n, dtype=torch.float64, device=dev)
    A = torch.randn(m, n + 1, dtype=torch.float64, device=dev)
    for _ in range(3):
        T = torch.mm(H, P)
        G = torch.mm(A.t(), A)
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    reps = 20
    e0.record()
    for _ in range(reps):
        T = torch.mm(H, P)
    e1.record()
    for _ in range(reps):
        G = torch.mm(A.t(), A)
    e2.record()
    torch.cuda.synchronize()
    t_hp = e0.elapsed_time(e1) / reps * 1e3
    t_g = e1.elapsed_time(e2) / reps * 1e3
    print("%-6s m %6d n %3d  T = H P: %7.1f us (%5.1f TFLOP/s)   G = A^T A: %7.1f us (%5.1f TFLOP/s)" % (
        name, m, n, t_hp, 2.0 * m * n * n / t_hp * 1e-6, t_g, 2.0 * m * (n + 1) ** 2 / t_g * 1e-6))
