"""triton_client_amd — the MI355X-native framework behind ``tritonclient``.

Sub-packages:
  ops/       HIP/CDNA4 kernels + HIP runtime bindings (ctypes over in-tree .so)
  models/    torch model definitions served by the bench server (DenseNet-121,
             BERT-large) — random-init, bf16, HIP-graph captured
  parallel/  multi-GPU fan-out (RCCL broadcast over xGMI, P2P star copies)
  perf/      perf_analyzer-equivalent load generator (Python driver + native)
  server/    in-repo KServe-v2 test & bench server (HTTP + gRPC)
  utils/     image codecs, timing helpers
"""
