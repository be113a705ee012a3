"""Every environment knob of the framework, in one table.

Two kinds:

* native: read by the host entry points of ``libtcamd_hip.so`` through the
  registry in ``csrc/runtime/knobs.hip`` (name, default and description live
  there: ``triton_client_amd.ops.hip.knobs()``); each is seeded from the
  environment once and can be switched in-process with
  ``hip.knob_set`` / ``with hip.knob(NAME=value)``.
* python / server: read once where noted (engine attributes can also be set on
  the object, which is how the tests switch them).

Each entry names the test that exercises it.  ``tests/test_knobs.py`` checks
that this table, the native registry, the sources (every ``TCAMD_*`` /
``TC_*`` / ``TCSERVE_*`` variable they read) and README's "Tuning knobs"
section agree, and that every named test exists.
"""

from collections import namedtuple

Knob = namedtuple("Knob", "name kind default where doc test")

_DF = "tests/test_densenet_fp32_gpu.py::"
_KN = "tests/test_knobs_gpu.py::"

KNOBS = [
    # ---- native (csrc/runtime/knobs.hip; doc strings there) ----
    Knob("TCAMD_X3_BM", "native", 0, "K8x 1x1 (densenet_x3.hip x3_plan)", "", _KN + "test_k8x_plan_knobs"),
    Knob("TCAMD_X3_SPLITK_BELOW", "native", 192, "K8x 1x1 split-K", "", _KN + "test_k8x_plan_knobs"),
    Knob("TCAMD_X3_MAX_SPLITS", "native", 4, "K8x 1x1 split-K cap", "", _KN + "test_k8x_plan_knobs"),
    Knob("TCAMD_X3_WS", "native", 1, "K8x warp-specialised 1x1", "", _KN + "test_k8x_plan_knobs"),
    Knob("TCAMD_X3_WS_MIN", "native", 16384, "K8x warp-specialised 1x1", "", _KN + "test_k8x_plan_knobs"),
    Knob("TCAMD_X3_STEM_BPC", "native", 2, "K10x stem grid", "", _KN + "test_stem_blocks_per_cu"),
    Knob("TCAMD_X3S_BLOCKS", "native", 384, "K13x 1x1 chunking", "", _KN + "test_k13x_chunking_and_split3"),
    Knob("TCAMD_X3S_MAX_CHUNKS", "native", 8, "K13x 1x1 chunking", "", _KN + "test_k13x_chunking_and_split3"),
    Knob("TCAMD_X3S_SPLIT3", "native", 1, "K13x 3x3 split", "", _KN + "test_k13x_chunking_and_split3"),
    Knob("TCAMD_PK_BIG_LIM", "native", (1 << 31) - (1 << 20), "K2 BYTES pack", "",
         "tests/test_kernels_gpu.py::test_pack_bytes_big_block_path"),
    Knob("TCAMD_K3_MODE", "native", 0, "K3 BYTES index", "", _KN + "test_k3_general_walk_mode"),
    Knob("TCAMD_K17_TM", "native", 0, "K17 GEMM tile height", "", "tests/test_gemm_gpu.py::test_k17_gemm_bf16_out"),
    Knob("TCAMD_K17_DYN", "native", 1, "K17 GEMM tile scheduling", "",
         "tests/test_gemm_gpu.py::test_k17_dynamic_schedule_every_tile_once"),
    # ---- python: fp32 DenseNet engine routing (models/densenet_fp32.py, engine attributes) ----
    Knob("TCAMD_X3_FUSE_MIN_TPB", "python", 1, "FP32DenseNet.fuse_min_tiles",
         "K11x for a block when every workgroup gets this many 64-pixel tiles; 0 = the K8x + K9x pair",
         _DF + "test_fp32_engine_routing_knobs"),
    Knob("TCAMD_X3_FUSE_BIGK_MIN_TPB", "python", 1, "FP32DenseNet.fuse_big_k_min_tiles",
         "K11x past K = 224 (to 480) from this many tiles per workgroup", _DF + "test_fp32_engine_routing_knobs"),
    Knob("TCAMD_X3_FUSE_V3", "python", 28, "FP32DenseNet.fuse_v3",
         "K11x v3 on blocks at least this wide (at >= 2 tiles per workgroup); 0 = v1 everywhere",
         _DF + "test_fp32_engine_routing_knobs"),
    Knob("TCAMD_X3_SMALL_M", "python", 1600, "FP32DenseNet.small_m",
         "K13x two-launch small-M layers up to this many pixels; 0 = off", _DF + "test_fp32_engine_routing_knobs"),
    Knob("TCAMD_X3_CHAIN", "python", 1, "FP32DenseNet.use_chain",
         "K13x chain (one launch per layer) for small-M blocks; 0 = two launches", _DF + "test_fp32_engine_routing_knobs"),
    Knob("TCAMD_X3_CHAIN_M", "python", 3136, "FP32DenseNet.chain_m",
         "largest block pixel count the chain takes", _DF + "test_fp32_engine_routing_knobs"),
    Knob("TCAMD_X3_SMALLF_MIN_BLOCKS", "python", "auto", "FP32DenseNet.smallf_min_blocks",
         "K14x for the 14x14 / 7x7 blocks from this many workgroups (images x row tiles); 0 = off; "
         "auto = 48 with concurrent streams (server instances), 64 on one",
         _DF + "test_fp32_engine_k14x_blocks_match_fp32_module"),
    Knob("TCAMD_X3_SMALLF_TILES", "python", 0, "FP32DenseNet.smallf_tiles",
         "K14x row tiles per image; 0 = the chip-filling choice (x3_small_tiles)",
         _DF + "test_fp32_engine_routing_knobs"),
    # ---- python: BERT ----
    Knob("TC_BERT_FUSED", "python", 1, "models/bert.py FUSED",
         "K11 / K12 fused kernels on the GPU; 0 = plain torch ops", "tests/test_bert_kernels_gpu.py::test_bert_fused_layers_match_torch_ops"),
    Knob("TC_BERT_GEMM", "python", "auto", "models/bert.py GEMM",
         "projection GEMMs: auto = the measured routing table (K18 where it beat hipBLASLt), ours = K18 / K17 "
         "everywhere, lib = hipBLASLt everywhere", "tests/test_gemm_gpu.py::test_bert_projection_routes"),
    Knob("TC_BERT_TUNED_GEMMS", "python", 0, "models/bert.py use_tuned_gemms",
         "TunableOp with the committed gfx950 solution table (process-wide; measured neutral)",
         _KN + "test_bert_tuned_gemm_table"),
    # ---- python: libraries, loading, serving ----
    Knob("TCAMD_HIP_LIB", "python", "", "ops/hip.py, csrc/cpp perf backend, image_client",
         "path of an alternative libtcamd_hip.so (A/B builds)", "tests/test_knobs.py::test_hip_lib_override_and_lazy_load"),
    Knob("TCAMD_LAZY_HIP", "python", 0, "ops/hip.py", "1 = load libtcamd_hip.so on first use, not at import",
         "tests/test_knobs.py::test_hip_lib_override_and_lazy_load"),
    Knob("TCAMD_NATIVE_EXEC", "python", 1, "server/gpu_models.py",
         "native C++ batch executor for graph models; 0 = the Python executor",
         "tests/test_executor_gpu.py::test_native_executor_matches_python_path"),
    Knob("TCAMD_BYTES_HOST_MAX", "python", 8192, "tritonclient/utils/hip_shared_memory",
         "BYTES set with bytes_path=auto: host codec up to this many elements, K2 above",
         "tests/test_knobs.py::test_bytes_auto_path_knobs"),
    Knob("TCAMD_BYTES_GET_DEVICE_MIN", "python", "", "tritonclient/utils/hip_shared_memory",
         "BYTES get with bytes_path=auto: K3 from this many elements (unset = host walk always)",
         "tests/test_knobs.py::test_bytes_auto_path_knobs"),
    Knob("TCAMD_FANOUT_FAULT", "python", "", "parallel/fanout.py",
         "fault injection: broadcast:RANK / p2p:RANK fails that rank's fan-out",
         "tests/test_distributed_cpu.py::test_time_fanout_agrees_on_a_one_rank_failure"),
    Knob("TC_ROCTX", "python", 0, "utils/roctx.py, csrc/cpp/src/trace.h",
         "1 = roctx ranges around perf windows and client calls", "tests/test_perf_analyzer.py::test_roctx_ranges_enabled_without_profiler"),
    Knob("TCSERVE_LIB", "python", "", "server/native_frontend.py", "path of an alternative libtcserve.so",
         "tests/test_knobs.py::test_tcserve_env_knobs"),
    Knob("TCSERVE_IO_THREADS", "python", 0, "server/native_frontend.py",
         "native front end event-loop threads; 0 = by CPU count", "tests/test_knobs.py::test_tcserve_env_knobs"),
    Knob("TCSERVE_HTTP", "python", 1, "server/app.py", "1 = the native front end also terminates REST",
         "tests/test_knobs.py::test_tcserve_env_knobs"),
    Knob("TCSERVE_STAGGER", "native-server", 1, "csrc/cpp/server/server.cc",
         "staggered dispatch of full batches across model instances; 0 = off",
         "tests/test_batch_policy.py::test_staggered_starts_of_full_batches"),
]

BY_NAME = {k.name: k for k in KNOBS}
