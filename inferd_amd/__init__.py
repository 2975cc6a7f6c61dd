"""inferd_amd -- MI355X-native (gfx950) Qwen3 layer-span engine behind InferD's span API.

The compute lives in libinferd_span.so (hand-written HIP kernels, C-ABI in
include/inferd_span.h).  Python here is the host side: the reference's node-facing
span API (partitioned_models), the gRPC-style session server (qwen3_server), the
span runtime / KV page table (runtime) and the multi-GPU pipeline (pipeline).
"""
__all__ = ["runtime", "partitioned_models", "qwen3_server", "pipeline"]
