"""perf_analyzer-equivalent load generation (Python driver; native tool in csrc/perf)."""
