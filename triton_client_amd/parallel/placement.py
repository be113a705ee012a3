"""Host placement for one-process-per-GPU runs: pin each rank (its server
child, the server's tcserve event loops and the native load generator's
threads) to CPU cores of its GPU's NUMA node.

SURVEY §2.8 / §7.4.7 turn the reference's one-worker-thread-per-client model
(reference src/c++/library/http_client.cc:2248-2348) into one event loop +
stream per GPU.  With 8 ranks on one host, 8 servers and 8 load generators
share the machine; unpinned, the scheduler moves their threads across sockets
and every request's host work pays remote-memory latency.  The plan:

  * the GPU of local rank r is the r-th GPU in the runtime's enumeration order
    (the KFD topology's GPU nodes by node id, the order ROCr and HIP use),
    filtered by ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES``;
  * its PCI address comes from the node's ``location_id`` / ``domain``, its
    NUMA node from ``/sys/bus/pci/devices/<bdf>/numa_node``;
  * the CPUs of that node (``/sys/devices/system/node/node<N>/cpulist``) that
    this process may use are split into equal disjoint slices among the local
    ranks whose GPUs sit on that node;
  * no NUMA information (node -1, a container without sysfs): the allowed CPUs
    are split evenly among all local ranks instead.

Nothing here touches the GPU (no HIP call), so the bench applies the plan
before it spawns the server: the child inherits the affinity.
"""

import os

KFD_NODES = "sys/class/kfd/kfd/topology/nodes"


def parse_cpulist(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpulist(cpus):
    """[0, 1, 2, 3, 8, 10, 11] -> '0-3,8,10-11'."""
    cpus = sorted(set(cpus))
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else "%d-%d" % (cpus[i], cpus[j]))
        i = j + 1
    return ",".join(out)


def _read(root, rel):
    try:
        with open(os.path.join(root, rel)) as f:
            return f.read()
    except OSError:
        return None


def _props(text):
    d = {}
    for line in (text or "").splitlines():
        parts = line.split()
        if len(parts) == 2:
            try:
                d[parts[0]] = int(parts[1])
            except ValueError:
                pass
    return d


def gpu_bdfs(root="/"):
    """PCI addresses of the GPUs in the runtime's enumeration order, after
    ``ROCR_VISIBLE_DEVICES`` and then ``HIP_VISIBLE_DEVICES`` (or its alias
    ``CUDA_VISIBLE_DEVICES`` when that is unset)."""
    base = os.path.join(root, KFD_NODES)
    try:
        ids = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return []
    out = []
    for n in ids:
        p = _props(_read(root, os.path.join(KFD_NODES, str(n), "properties")))
        if p.get("simd_count", 0) <= 0:  # a CPU node
            continue
        loc, dom = p.get("location_id", 0), p.get("domain", 0)
        out.append("%04x:%02x:%02x.%x" % (dom, (loc >> 8) & 0xFF, (loc >> 3) & 0x1F, loc & 0x7))
    # ROCR filters first; then HIP applies HIP_VISIBLE_DEVICES, and
    # CUDA_VISIBLE_DEVICES only as its alias when HIP_VISIBLE_DEVICES is unset
    # (never both: a second filter would map a rank to the wrong GPU)
    hip_var = "HIP_VISIBLE_DEVICES" if os.environ.get("HIP_VISIBLE_DEVICES") else "CUDA_VISIBLE_DEVICES"
    for var in ("ROCR_VISIBLE_DEVICES", hip_var):
        vis = os.environ.get(var)
        if vis:
            try:
                out = [out[int(v)] for v in vis.split(",") if v.strip() != "" and int(v) < len(out)]
            except ValueError:  # UUID lists: leave the order alone
                pass
    return out


def numa_node(bdf, root="/"):
    v = _read(root, os.path.join("sys/bus/pci/devices", bdf, "numa_node"))
    try:
        return int(v) if v is not None else -1
    except ValueError:
        return -1


def node_cpus(node, root="/"):
    v = _read(root, "sys/devices/system/node/node%d/cpulist" % node)
    return parse_cpulist(v) if v else []


def plan(local_rank, local_world, root="/", allowed=None):
    """The CPU set of ``local_rank`` among ``local_world`` ranks on this host.
    Returns {"cpus": [...], "cpulist": str, "numa_node": int, "bdf": str|None,
    "ranks_on_node": int, "source": "numa" | "even-split"}."""
    allowed = sorted(allowed if allowed is not None else os.sched_getaffinity(0))
    bdfs = gpu_bdfs(root)
    nodes = [numa_node(b, root) for b in bdfs[:local_world]]
    bdf = bdfs[local_rank] if local_rank < len(bdfs) else None
    node = nodes[local_rank] if local_rank < len(nodes) else -1
    if node >= 0:
        cpus = [c for c in node_cpus(node, root) if c in set(allowed)]
        peers = [r for r in range(local_world) if r < len(nodes) and nodes[r] == node]
        if cpus and local_rank in peers:
            k, n = peers.index(local_rank), len(peers)
            share = _slice(cpus, k, n)
            if share:
                return {"cpus": share, "cpulist": format_cpulist(share), "numa_node": node, "bdf": bdf,
                        "ranks_on_node": n, "source": "numa"}
    share = _slice(allowed, local_rank, max(local_world, 1))
    return {"cpus": share, "cpulist": format_cpulist(share), "numa_node": node, "bdf": bdf,
            "ranks_on_node": local_world, "source": "even-split"}


def _slice(cpus, k, n):
    """The k-th of n near-equal contiguous slices of cpus (every CPU in exactly
    one slice; with more ranks than CPUs a rank shares its neighbour's CPU)."""
    if not cpus:
        return []
    if n > len(cpus):
        return [cpus[k % len(cpus)]]
    lo = len(cpus) * k // n
    hi = len(cpus) * (k + 1) // n
    return cpus[lo:hi]


def apply(p):
    """Pin this process (and every thread and child it starts from now on)
    to the plan's CPUs.  Returns the plan with ``applied`` set."""
    p = dict(p)
    try:
        os.sched_setaffinity(0, p["cpus"])
        p["applied"] = True
    except (OSError, ValueError) as e:
        p["applied"] = False
        p["error"] = str(e)
    return p
