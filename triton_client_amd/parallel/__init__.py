"""Multi-GPU fan-out over RCCL / xGMI peer copies (one process per GPU)."""
