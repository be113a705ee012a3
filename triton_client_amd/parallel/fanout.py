"""Multi-GPU fan-out of the shared synthetic input batch.

One process per GPU (torch.distributed, backend "nccl" == RCCL on ROCm).
Rank 0 generates the synthetic batch once on its GPU (K1 synth_fill) and the
batch is replicated into every rank's HIP shared-memory input region:

* ``rccl``  — X1: ``dist.broadcast`` straight into the region (the region is
  exposed to torch through a zero-copy kDLROCM DLPack view).
* ``p2p``   — X2: a one-hop star over xGMI: ranks all-gather their regions'
  IPC handles, rank 0 opens them and issues one hipMemcpyAsync per peer on
  its own stream (each copy uses the direct rank0->peer link; no ring hops).
  Ranks then barrier.
* ``local`` — every rank generates the identical data itself (K1 is a pure
  function of (seed, offset)), used when no process group exists.

For a few-MB batch the broadcast is latency-bound (densenet bs=8: 4.8 MB is
~31 us at ~153 GB/s per link), so the star pays one hop where a ring pays 7.
"""

import numpy as np

from triton_client_amd.utils import roctx


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def region_tensor(region, nbytes):
    """torch uint8 tensor aliasing the first ``nbytes`` of a HIP shm region."""
    import torch

    from tritonclient.utils import hip_shared_memory as hipshm

    view = hipshm.as_shared_memory_tensor(region, "UINT8", [nbytes])
    return torch.from_dlpack(view)


def fill_and_fanout(region, datatype, n_elems, seed=0, mode="random", lo=0.0, hi=1.0, method="rccl"):
    """Fill ``region`` on rank 0 and replicate to every rank. Returns method used."""
    from tritonclient.utils import hip_shared_memory as hipshm
    from triton_client_amd.ops import dtypes

    dist = _dist()
    nbytes = n_elems * dtypes.SIZES[datatype]
    if dist is None or dist.get_world_size() == 1:
        hipshm.fill_synthetic_data(region, datatype, n_elems, mode, lo, hi, seed)
        return "local"
    rank = dist.get_rank()
    if method == "local":
        hipshm.fill_synthetic_data(region, datatype, n_elems, mode, lo, hi, seed)
        dist.barrier()
        return "local"
    if rank == 0:
        hipshm.fill_synthetic_data(region, datatype, n_elems, mode, lo, hi, seed)
    if method == "rccl":
        import torch

        t = region_tensor(region, nbytes)
        try:
            with roctx.range("fanout.rccl_broadcast bytes=%d" % t.numel()):
                dist.broadcast(t, src=0)
            torch.cuda.synchronize()
            return "rccl"
        except Exception as e:  # noqa: BLE001
            # the Philox fill is deterministic: every rank can produce the
            # same replica itself (the caller still verifies the replicas)
            import sys

            print("[fanout] rccl broadcast failed (%s); filling locally" % str(e)[:200], file=sys.stderr)
            hipshm.fill_synthetic_data(region, datatype, n_elems, mode, lo, hi, seed)
            torch.cuda.synchronize()
            return "local (rccl broadcast failed)"
    if method == "p2p":
        with roctx.range("fanout.p2p_star bytes=%d" % nbytes):
            return _p2p_star(region, nbytes, dist)
    raise ValueError("unknown fan-out method %s" % method)


def _sync_all(dist):
    import torch

    if torch.cuda.is_available():
        torch.cuda.synchronize()
    dist.barrier()


def replicate(region, nbytes, method):
    """Copy rank 0's first ``nbytes`` of ``region`` into every rank's region
    (no refill).  rccl: one broadcast collective (X1); p2p: the xGMI one-hop
    star from rank 0 (X2); host: staged through host memory and a gloo/CPU
    broadcast (the rehearsal path when several ranks share one GPU)."""
    dist = _dist()
    if dist is None or dist.get_world_size() == 1:
        return "local"
    if method == "rccl":
        t = region_tensor(region, nbytes)
        with roctx.range("fanout.rccl_broadcast bytes=%d" % nbytes):
            dist.broadcast(t, src=0)
        return "rccl"
    if method == "p2p":
        with roctx.range("fanout.p2p_star bytes=%d" % nbytes):
            return _p2p_star(region, nbytes, dist)
    if method == "host":
        import torch

        t = region_tensor(region, nbytes)
        h = t.cpu() if dist.get_rank() == 0 else torch.empty(nbytes, dtype=torch.uint8)
        dist.broadcast(h, src=0)
        t.copy_(h.to(t.device))
        return "host"
    raise ValueError("unknown fan-out method %s" % method)


def time_fanout(region, nbytes, methods, reps=5):
    """Time each fan-out method replicating the (already filled) region:
    median over ``reps`` of barrier -> replicate -> device sync -> barrier,
    MAX over ranks.  Returns {method: {"us", "GBps_per_peer", "bytes"}} or an
    {"error": ...} entry for a method this process group cannot run."""
    import time

    dist = _dist()
    out = {}
    if dist is None or dist.get_world_size() == 1:
        return out
    for m in methods:
        ts = []
        try:
            for _ in range(reps + 1):
                _sync_all(dist)
                t0 = time.perf_counter()
                replicate(region, nbytes, m)
                _sync_all(dist)
                ts.append(time.perf_counter() - t0)
        except Exception as e:  # noqa: BLE001 - reported in the JSON, the run goes on
            out[m] = {"error": str(e)[:200]}
            try:
                dist.barrier()
            except Exception:
                pass
            continue
        med = float(np.median(ts[1:]))
        med = max_over_ranks(med)
        out[m] = {"us": round(med * 1e6, 1), "GBps_per_peer": round(nbytes / med / 1e9, 2), "bytes": int(nbytes)}
    return out


def _p2p_star(region, nbytes, dist):
    from tritonclient.utils import hip_shared_memory as hipshm  # noqa: F401
    from triton_client_amd.ops import hip

    rank = dist.get_rank()
    world = dist.get_world_size()
    handles = [None] * world
    dist.all_gather_object(handles, (region._device_id, region._hip_shm_handle))
    if rank == 0:
        src_dev = region._device_id
        streams = []
        opened = []
        try:
            for peer in range(1, world):
                dev, h = handles[peer]
                try:
                    hip.enable_peer(src_dev, dev)
                except Exception:
                    pass  # copies still work through the runtime's staging path
                ptr = hip.ipc_open(h, src_dev)
                opened.append(ptr)
                s = hip.Stream(src_dev)
                streams.append(s)
                hip.memcpy_async(ptr, region._base_addr, nbytes, s.handle)
            for s in streams:
                s.synchronize()
        finally:
            for s in streams:
                s.close()
            for p in opened:
                hip.ipc_close(p, src_dev)
    dist.barrier()
    return "p2p"


def fanout_host(buf, src=0):
    """Replicate a host buffer (e.g. a system shared-memory region's numpy
    view) from rank ``src`` to every rank with one collective broadcast
    (gloo on CPU hosts, or RCCL when the process group is nccl — the tensor is
    then staged through the GPU)."""
    import torch

    dist = _dist()
    if dist is None or dist.get_world_size() == 1:
        return "local"
    t = torch.from_numpy(np.asarray(buf).view(np.uint8).reshape(-1))
    if dist.get_backend() == "gloo":
        dist.broadcast(t, src=src)
    else:
        d = t.cuda()
        dist.broadcast(d, src=src)
        t.copy_(d.cpu())
    return dist.get_backend()


def verify_host_replicas(buf, sample=4096):
    """Every rank checks a strided sample of a host buffer against rank 0's."""
    import torch

    dist = _dist()
    if dist is None:
        return True
    a = np.asarray(buf).view(np.uint8).reshape(-1)
    idx = np.linspace(0, a.size - 1, min(sample, a.size)).astype(np.int64)
    s = torch.from_numpy(a[idx].astype(np.int64))
    ref = s.clone()
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    ref = ref.to(dev)
    dist.broadcast(ref, src=0)
    flag = torch.tensor([1 if torch.equal(s, ref.cpu()) else 0], device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def verify_replicas(region, nbytes, sample=4096):
    """Every rank checks a strided sample of its region against rank 0's."""
    import torch

    dist = _dist()
    t = region_tensor(region, nbytes)
    idx = torch.linspace(0, nbytes - 1, min(sample, nbytes), device=t.device).long()
    s = t[idx].to(torch.int64)
    if dist is None:
        return True
    if dist.get_backend() == "gloo":  # rehearsal: collectives on host copies
        s = s.cpu()
    ref = s.clone()
    dist.broadcast(ref, src=0)
    ok = torch.equal(s, ref)
    flag = torch.tensor([1 if ok else 0], device=s.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def max_over_ranks(value):
    """MAX of a python float across ranks (identity without a process group)."""
    dist = _dist()
    if dist is None:
        return value
    import torch

    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    if dist.get_backend() == "gloo":
        dev = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_arrays(arr):
    """Concatenate a 1-D numpy int64 array from all ranks (on every rank)."""
    dist = _dist()
    if dist is None:
        return arr
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, np.asarray(arr))
    return np.concatenate(out) if out else arr
