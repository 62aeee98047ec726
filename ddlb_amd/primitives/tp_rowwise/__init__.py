"""TP-Rowwise (GEMM -> reduce-scatter, sequence parallel) implementations."""
