"""numpy reference of the K1 synth_fill Philox4x32-10 stream (csrc/kernels/synth.hip)."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = [np.asarray(x, dtype=np.uint64) for x in (c0, c1, c2, c3)]
    k0 = np.uint64(k0)
    k1 = np.uint64(k1)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK, lo1, (hi0 ^ c3 ^ k1) & MASK, lo0
        k0 = (k0 + np.uint64(W0)) & MASK
        k1 = (k1 + np.uint64(W1)) & MASK
    return [x.astype(np.uint32) for x in (c0, c1, c2, c3)]


def raw_u32(n_elems, elem_size, seed=0, stream_id=0):
    """The raw uint32 feeding element i (same mapping as fill_chunk)."""
    per_chunk = 16 // elem_size
    n_chunks = (n_elems + per_chunk - 1) // per_chunk
    chunk = np.arange(n_chunks, dtype=np.uint64)
    subs = (per_chunk + 3) // 4
    out = np.empty((n_chunks, subs * 4), dtype=np.uint32)
    for s in range(subs):
        r = philox(chunk & MASK, chunk >> np.uint64(32), np.uint64(s ^ (stream_id & 0xFFFFFFFF)),
                   np.uint64(stream_id >> 32), seed & 0xFFFFFFFF, seed >> 32)
        out[:, 4 * s : 4 * s + 4] = np.stack(r, axis=1)
    return out[:, :per_chunk].reshape(-1)[:n_elems]


def uniform_f32(n, lo, hi, seed=0, stream_id=0):
    u = (raw_u32(n, 4, seed, stream_id) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return (lo + u.astype(np.float64) * (hi - lo)).astype(np.float32)
