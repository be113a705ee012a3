"""Multi-process (one process per "GPU") rehearsal of bench.py's distributed
flow on CPU with the gloo backend, world_size 2: every rank runs its own
server, rank 0's synthetic batch is fanned out into every rank's shared
memory region by a collective, each rank drives its server with the native
perf engine, and the job takes the MAX elapsed over ranks."""

import json
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from triton_client_amd.parallel import fanout
    from triton_client_amd.perf.native import PerfSession, available
    from triton_client_amd.server import ServerHandle
    import tritonclient.grpc as grpcclient
    from tritonclient.utils import shared_memory as shm

    res = {"rank": rank}
    h = ServerHandle(models=None).start()
    key = "/dist_in_%d_%d" % (os.getpid(), rank)
    region = shm.create_shared_memory_region("dist_in", key, 2 * 64)
    try:
        view = np.ndarray((32,), dtype=np.int32, buffer=shm.get_contents_as_numpy(region, np.uint8, [128]))
        if rank == 0:
            view[:] = np.arange(32, dtype=np.int32) * 7
        res["method"] = fanout.fanout_host(view)
        res["replicas_ok"] = fanout.verify_host_replicas(view)
        res["data"] = view.copy().tolist()
        c = grpcclient.InferenceServerClient(h.grpc_url)
        c.register_system_shared_memory("dist_in", key, 128)
        if available():
            with PerfSession(["-m", "add_sub_batched", "-i", "grpc", "-u", h.grpc_url, "-b", "1",
                              "--shared-memory", "system", "--shared-memory-input", "INPUT0=dist_in",
                              "--shared-memory-input", "INPUT1=dist_in", "--concurrency-range", "4"]) as perf:
                perf.run_fixed(4, 20)
                dist.barrier()
                lat, el = perf.run_fixed(4, 200)
                dist.barrier()
            res["elapsed"] = el
            res["elapsed_max"] = fanout.max_over_ranks(el)
            res["n_lat_all"] = int(fanout.gather_arrays(np.asarray(lat, dtype=np.int64)).size)
        c.unregister_system_shared_memory()
    finally:
        shm.destroy_shared_memory_region(region)
        h.stop()
        dist.destroy_process_group()
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump(res, f)


def test_two_rank_fanout_and_perf(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    results = []
    for r in range(world):
        with open(os.path.join(tmp_path, "rank%d.json" % r)) as f:
            results.append(json.load(f))
    for r in results:
        assert r["method"] == "gloo"
        assert r["replicas_ok"]
        assert r["data"] == (np.arange(32) * 7).tolist()
    if "elapsed" in results[0]:
        assert results[0]["elapsed_max"] == results[1]["elapsed_max"] == max(r["elapsed"] for r in results)
        assert results[0]["n_lat_all"] == 400
