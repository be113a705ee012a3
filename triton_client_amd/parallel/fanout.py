"""Multi-GPU fan-out of the shared synthetic input batch.

One process per GPU (torch.distributed, backend "nccl" == RCCL on ROCm).
Rank 0 generates the synthetic batch once on its GPU (K1 synth_fill) and the
batch is replicated into every rank's HIP shared-memory input region:

* ``rccl``  — X1: ``dist.broadcast`` straight into the region (the region is
  exposed to torch through a zero-copy kDLROCM DLPack view).
* ``p2p``   — X2: a one-hop star over xGMI in which every destination
  PULLS: rank 0 broadcasts its region's IPC handle, each other rank opens it
  and copies rank 0's bytes into its own region with one hipMemcpyAsync on
  its own stream -- its own GPU's copy engines over its own direct link to
  rank 0 (no ring hops, and rank 0's engines are not the serial point of
  seven copies).  Ranks then barrier.  The native load generator's star
  (csrc/cpp/perf/multigpu.cc) pulls the same way.
* ``local`` — every rank generates the identical data itself (K1 is a pure
  function of (seed, offset)), used when no process group exists.

For a few-MB batch the broadcast is latency-bound (densenet bs=8: 4.8 MB is
~31 us at ~153 GB/s per link), so the star pays one hop where a ring pays 7.
"""

import os
import sys

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


def _fill(region, datatype, n_elems, mode, lo, hi, seed):
    from tritonclient.utils import hip_shared_memory as hipshm

    hipshm.fill_synthetic_data(region, datatype, n_elems, mode, lo, hi, seed)


def _device_sync():
    import torch

    if torch.cuda.is_available():
        torch.cuda.synchronize()


_CPU_GROUP = []


def cpu_group(timeout_s=300):
    """A gloo group over the same ranks, for control-plane agreement.  An RCCL
    failure must not be voted on over the communicator that just failed: a
    poisoned communicator hangs or pairs the vote with the wrong collective on
    the other ranks.  Creating a group is itself collective, so every rank calls
    this once right after init_process_group (bench.py does).  Returns None
    (= the default group) when the default group already is gloo."""
    dist = _dist()
    if dist is None or dist.get_backend() == "gloo":
        return None
    if not _CPU_GROUP:
        import datetime

        _CPU_GROUP.append(dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s)))
    return _CPU_GROUP[0]


def all_ok(ok):
    """True on every rank iff ``ok`` is true on every rank (MIN over the gloo
    control group; also a barrier)."""
    dist = _dist()
    if dist is None or dist.get_world_size() == 1:
        return bool(ok)
    import torch

    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=cpu_group())
    return bool(t.item())


def _fault(point):
    """Test hook: TCAMD_FANOUT_FAULT=<point>:<rank,rank..> raises after the
    collective at ``point`` on the listed ranks (an NCCL error surfaces at the
    next synchronize, after the call was issued on every rank)."""
    spec = os.environ.get("TCAMD_FANOUT_FAULT", "")
    if not spec or ":" not in spec:
        return
    where, ranks = spec.split(":", 1)
    dist = _dist()
    if where == point and dist is not None and str(dist.get_rank()) in ranks.split(","):
        raise RuntimeError("injected %s fault on rank %d" % (point, dist.get_rank()))


def fill_and_fanout(region, datatype, n_elems, seed=0, mode="random", lo=0.0, hi=1.0, method="rccl",
                    fallback=None):
    """Fill ``region`` on rank 0 and replicate to every rank.  Returns the
    method used.

    A failed RCCL broadcast raises (the caller exits non-zero with the error):
    the north star's fan-out must not be skipped quietly.  ``fallback="local"``
    (bench.py ``--fanout-fallback local``) instead has every rank agree on the
    broadcast's outcome over the gloo control group and, if any rank failed,
    refill locally (K1 is a pure function of (seed, offset)); the method is then
    labelled ``"local (fallback: rccl broadcast failed)"`` and the replicas must
    be verified over the control group (``verify_replicas(..., over_cpu=True)``)."""
    from triton_client_amd.ops import dtypes

    dist = _dist()
    nbytes = n_elems * dtypes.SIZES[datatype]
    if dist is None or dist.get_world_size() == 1:
        _fill(region, datatype, n_elems, mode, lo, hi, seed)
        return "local"
    rank = dist.get_rank()
    if method == "local":
        _fill(region, datatype, n_elems, mode, lo, hi, seed)
        dist.barrier()
        return "local"
    if fallback not in (None, "none", "local"):
        raise ValueError("unknown fan-out fallback %s" % fallback)
    if rank == 0:
        _fill(region, datatype, n_elems, mode, lo, hi, seed)
    if method == "rccl":
        t = region_tensor(region, nbytes)
        err = None
        try:
            with roctx.range("fanout.rccl_broadcast bytes=%d" % t.numel()):
                dist.broadcast(t, src=0)
            _fault("broadcast")
            _device_sync()
        except Exception as e:  # noqa: BLE001 - re-raised below unless the fallback is asked for
            err = e
        if fallback != "local":
            if err is not None:
                raise RuntimeError("RCCL broadcast of the synthetic batch failed on rank %d: %s"
                                   % (rank, err)) from err
            return "rccl"
        if all_ok(err is None):
            return "rccl"
        if err is not None:
            print("[fanout] rank %d: rccl broadcast failed (%s)" % (rank, str(err)[:200]), file=sys.stderr)
        _fill(region, datatype, n_elems, mode, lo, hi, seed)
        _device_sync()
        return LOCAL_FALLBACK
    if method == "p2p":
        with roctx.range("fanout.p2p_star bytes=%d" % nbytes):
            return _p2p_star(region, nbytes, dist)
    raise ValueError("unknown fan-out method %s" % method)


LOCAL_FALLBACK = "local (fallback: rccl broadcast failed)"


def _sync_all(dist):
    _device_sync()
    dist.barrier(group=cpu_group())


def barrier():
    """Barrier over the gloo control group (no-op without a process group):
    the bench's control plane never rides on the RCCL communicator, so an RCCL
    fallback run can still bracket, aggregate and report."""
    dist = _dist()
    if dist is not None:
        dist.barrier(group=cpu_group())


def replicate(region, nbytes, method, errors=None):
    """Copy rank 0's first ``nbytes`` of ``region`` into every rank's region
    (no refill).  rccl: one broadcast collective (X1); p2p: the xGMI one-hop
    star from rank 0 (X2); host: staged through host memory and a gloo/CPU
    broadcast (the rehearsal path when several ranks share one GPU).

    A p2p copy failure on rank 0 is caught there (every rank still reaches the
    star's closing barrier): with an ``errors`` list it is appended for the
    caller to agree on later, otherwise the ranks agree now over the gloo control
    group and all raise together."""
    dist = _dist()
    if dist is None or dist.get_world_size() == 1:
        return "local"
    if method == "rccl":
        t = region_tensor(region, nbytes)
        with roctx.range("fanout.rccl_broadcast bytes=%d" % nbytes):
            dist.broadcast(t, src=0)
        _fault("broadcast")
        return "rccl"
    if method == "p2p":
        with roctx.range("fanout.p2p_star bytes=%d" % nbytes):
            err = _p2p_copy(region, nbytes, dist)
        if errors is not None:
            if err is not None:
                errors.append(err)
        elif not all_ok(err is None):
            raise RuntimeError("p2p fan-out failed: %s" % (err if err is not None else "on another rank"))
        return "p2p"
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
    MAX over ranks.  Returns {method: {"us", "GBps_per_peer", "bytes"}}; a p2p
    method whose copies failed on any rank gets an agreed {"error": ...} entry
    on every rank (the ranks never leave the common collective sequence: the
    failure is caught where it happens and voted on over the gloo control
    group).  A collective that raises (RCCL) propagates: the communicator is
    unusable after it, and the run must fail loudly."""
    import time

    dist = _dist()
    out = {}
    if dist is None or dist.get_world_size() == 1:
        return out
    for m in methods:
        ts, errors = [], []
        for _ in range(reps + 1):
            _sync_all(dist)
            t0 = time.perf_counter()
            replicate(region, nbytes, m, errors=errors)
            _sync_all(dist)
            ts.append(time.perf_counter() - t0)
        if not all_ok(not errors):
            out[m] = {"error": str(errors[0])[:200] if errors else "failed on another rank"}
            continue
        med = float(np.median(ts[1:]))
        med = max_over_ranks(med)
        out[m] = {"us": round(med * 1e6, 1), "GBps_per_peer": round(nbytes / med / 1e9, 2), "bytes": int(nbytes)}
        if m == "p2p":
            # every destination timed its own pull (last rep): per-peer copy
            # time and whether its link to rank 0 had peer access
            peers = [None] * dist.get_world_size()
            dist.all_gather_object(peers, dict(_LAST_PULL), group=cpu_group())
            out[m]["per_peer"] = {str(r): {"us": round(p["us"], 1), "peer_access": p["peer_access"]}
                                  for r, p in enumerate(peers) if r != 0 and p}
            acc = [p["peer_access"] for r, p in enumerate(peers) if r != 0 and p]
            ok = all(a is not False for a in acc)
            out[m]["peer_access"] = ok if any(a is not None for a in acc) else None
            if not ok:
                out[m]["note"] = ("hipDeviceEnablePeerAccess failed for a peer: its pull ran over the "
                                  "runtime's staging path, not the xGMI star")
            elif out[m]["peer_access"] is None:
                out[m]["note"] = "every rank shares rank 0's GPU (rehearsal): no xGMI link was used"
    return out


def fanout_errors(timings):
    """{method: error} of a time_fanout result (surfaced at the top level of
    the bench JSON)."""
    return {m: v["error"] for m, v in (timings or {}).items() if "error" in v}


# this rank's last X2 pull: {"us": copy time, "peer_access": bool or None
# (None: same device as rank 0, no link to enable)}
_LAST_PULL = {}


def _pull_copy(region, src_dev, handle, nbytes):
    """A destination rank's half of the X2 star: open rank 0's region (IPC
    handle) on this rank's device and copy it into this rank's region on a
    stream of its own -- this GPU's copy engines, over its direct link to rank
    0.  ``hipDeviceEnablePeerAccess`` failing is recorded (the runtime then
    stages the copy, and the timing is not the xGMI star) and reported as
    ``peer_access: false``.  Returns (microseconds, peer_access)."""
    import time

    from tritonclient.utils import hip_shared_memory as hipshm  # noqa: F401
    from triton_client_amd.ops import hip

    dev = region._device_id
    access = None
    if dev != src_dev:
        try:
            hip.enable_peer(dev, src_dev)
            access = True
        except Exception as e:  # noqa: BLE001 - recorded and reported, never swallowed
            access = False
            print("[fanout] hipDeviceEnablePeerAccess(%d -> %d) failed: %s" % (dev, src_dev, str(e)[:200]),
                  file=sys.stderr)
    ptr = hip.ipc_open(handle, dev)
    s = None
    try:
        s = hip.Stream(dev)
        t0 = time.perf_counter()
        hip.memcpy_async(region._base_addr, ptr, nbytes, s.handle)
        s.synchronize()
        us = (time.perf_counter() - t0) * 1e6
    finally:
        if s is not None:
            s.close()
        hip.ipc_close(ptr, dev)
    return us, access


def _p2p_copy(region, nbytes, dist):
    """The X2 star (pull).  Returns this rank's exception (its copy failure, or
    an injected fault) or None; every rank reaches the closing barrier either
    way, so the collective sequence stays aligned and the caller can agree on
    the outcome."""
    rank = dist.get_rank()
    src = [(region._device_id, region._hip_shm_handle) if rank == 0 else None]
    dist.broadcast_object_list(src, src=0, group=cpu_group())
    err = None
    _LAST_PULL.clear()
    if rank != 0:
        try:
            us, access = _pull_copy(region, src[0][0], src[0][1], nbytes)
            _LAST_PULL.update({"us": us, "peer_access": access})
        except Exception as e:  # noqa: BLE001 - agreed on by the caller
            err = e
    try:
        _fault("p2p")  # test hook: recorded like a real copy error, before the barrier
    except RuntimeError as e:
        err = err or e
    dist.barrier(group=cpu_group())
    return err


def _p2p_star(region, nbytes, dist):
    err = _p2p_copy(region, nbytes, dist)
    if not all_ok(err is None):
        raise RuntimeError("p2p fan-out failed: %s" % (err if err is not None else "on another rank"))
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


def sample_positions(nbytes, sample=4096, device="cpu"):
    """``min(sample, nbytes)`` evenly spread byte positions in [0, nbytes),
    first and last included, in int64 arithmetic (a float32 linspace rounds
    the last position of a > 16 MiB region past its end: an out-of-bounds
    device read)."""
    import torch

    n = min(sample, nbytes)
    return torch.arange(n, device=device, dtype=torch.int64) * (nbytes - 1) // max(n - 1, 1)


def verify_replicas(region, nbytes, sample=4096, over_cpu=False):
    """Every rank checks a strided sample of its region against rank 0's
    (``over_cpu``: over the gloo control group, after an RCCL fallback)."""
    import torch

    dist = _dist()
    if dist is None:
        return True
    t = region_tensor(region, nbytes)
    idx = sample_positions(nbytes, sample, t.device)
    s = t[idx].to(torch.int64)
    group = None
    if over_cpu:
        group = cpu_group()
        s = s.cpu()
    elif dist.get_backend() == "gloo":  # rehearsal: collectives on host copies
        s = s.cpu()
    ref = s.clone()
    dist.broadcast(ref, src=0, group=group)
    ok = torch.equal(s, ref)
    flag = torch.tensor([1 if ok else 0], device=s.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item())


def max_over_ranks(value):
    """MAX of a python float across ranks (identity without a process group)."""
    dist = _dist()
    if dist is None:
        return value
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=cpu_group())
    return float(t.item())


def gather_arrays(arr):
    """Concatenate a 1-D numpy int64 array from all ranks (on every rank)."""
    dist = _dist()
    if dist is None:
        return arr
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, np.asarray(arr), group=cpu_group())
    return np.concatenate(out) if out else arr


def gather_objects(obj):
    """[obj of rank 0, obj of rank 1, ...] on every rank ([obj] without a process group)."""
    dist = _dist()
    if dist is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj, group=cpu_group())
    return out
