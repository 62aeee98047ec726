"""TP-Columnwise (all-gather -> GEMM) implementations: compute_only, pytorch, native."""
