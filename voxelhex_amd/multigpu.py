"""Screen-tile sharding of a frame across ranks (one process per GPU) and the gather to rank 0.

The frame is cut into T x T tiles in raster order; rank r traces tiles r, r + world, r + 2*world, ... into one
contiguous tile-major buffer (VHX_LAYOUT_TILES: the j-th tile of the rank at [j*T*T, (j+1)*T*T), row-major inside,
zeros past the frame edge). Rank 0 gathers the buffers (RCCL over xGMI with the nccl backend; gloo on CPU) and
scatters them into the framebuffer (vhx_untile_rgba on the GPU; untile_numpy is the host restatement used by tests).
"""
import ctypes

import numpy as np

from . import _native as N


def tile_grid(width, height, T):
    return (width + T - 1) // T, (height + T - 1) // T


def tiles_per_rank(width, height, T, world):
    tx, ty = tile_grid(width, height, T)
    return (tx * ty + world - 1) // world


def rank_tiles(width, height, T, rank, world):
    tx, ty = tile_grid(width, height, T)
    return list(range(rank, tx * ty, world))


def tile_rect(tile, width, height, T):
    tx, _ = tile_grid(width, height, T)
    x0, y0 = (tile % tx) * T, (tile // tx) * T
    return x0, y0, min(T, width - x0), min(T, height - y0)


def rank_rays(width, height, T, rank, world):
    return sum(w * h for _, _, w, h in (tile_rect(t, width, height, T) for t in rank_tiles(width, height, T, rank, world)))


def tile_plan(nranks, root_slots, T, width, height, rank):
    """vhx_mgpu_tile_plan (the C deal vhx_mgpu_render uses; pure, no device): dict with tiles_x, tiles_y, tiles, slots,
    tiles_per_slot, first_slot, slot_count."""
    p = N.TilePlan()
    rc = N.lib().vhx_mgpu_tile_plan(nranks, root_slots, T, width, height, rank, ctypes.byref(p))
    if rc != N.VHX_OK:
        raise ValueError(f"vhx_mgpu_tile_plan({nranks}, {root_slots}, {T}, {width}, {height}, {rank}) = {rc}")
    return {name: getattr(p, name) for name, _ in N.TilePlan._fields_ if name != "reserved"}


def untile_numpy(gathered, ranks, per_rank, T, width, height):
    """Host restatement of k_untile_rgba: gathered = concatenation over ranks of per_rank*T*T pixels."""
    fb = np.zeros(width * height, gathered.dtype)
    for r in range(ranks):
        for j, tile in enumerate(range(r, tile_grid(width, height, T)[0] * tile_grid(width, height, T)[1], ranks)):
            x0, y0, w, h = tile_rect(tile, width, height, T)
            blk = gathered[(r * per_rank + j) * T * T:(r * per_rank + j + 1) * T * T].reshape(T, T)
            fb.reshape(height, width)[y0:y0 + h, x0:x0 + w] = blk[:h, :w]
    return fb


def untile_planes_numpy(gathered, planes, ranks, per_rank, T, width, height):
    """Host restatement of k_untile_planes (vhx_untile_frame): rank r's part of `gathered` holds `planes` planes of
    per_rank*T*T words ([RGBA | depth] for planes = 2); returns one framebuffer per plane."""
    n = per_rank * T * T
    g = np.asarray(gathered).reshape(ranks, planes, n)
    return [untile_numpy(np.ascontiguousarray(g[:, p, :]).reshape(-1), ranks, per_rank, T, width, height)
            for p in range(planes)]


class GatherPipeline:
    """Per-frame gather of every rank's tile buffer to rank 0 and the untile there, overlapped with the next frame.

    Two output buffers alternate: frame k is traced into `out_buffer()`, then `submit()` first completes frame k-1's
    gather (the caller's stream waits for it) and untiles it, then starts frame k's gather asynchronously (RCCL runs
    on its own stream), so frame k+1's trace overlaps frame k's transfer. Buffer reuse is stream-ordered: frame k+2
    writes frame k's buffer only after submit(k+1) waited for frame k's gather. `drain()` completes the last frame.
    With overlap=False each submit gathers and untiles its frame before returning to the caller's stream order.

    untile(gathered, slot) scatters rank 0's gathered buffer (world * n_out pixels, rank-major) into the framebuffer.
    host_staging: the gather runs over host memory (gloo rehearsal of the multi-GPU path on one GPU; synchronous).
    """

    def __init__(self, n_out, world, rank, dist, device, untile, overlap=True, host_staging=False):
        import torch
        self.world, self.rank, self.dist, self.untile = world, rank, dist, untile
        self.overlap = overlap and not host_staging
        self.host_staging = host_staging
        self.bufs = [torch.zeros(n_out, dtype=torch.int32, device=device) for _ in range(2)]
        self.big = self.parts = None
        if rank == 0:
            self.big = [torch.zeros(world * n_out, dtype=torch.int32, device=device) for _ in range(2)]
            self.parts = [list(b.chunk(world)) for b in self.big]  # views: the gather writes in place, no cat
        self.k = 0
        self.pending = None  # (work handle, slot) of the frame whose gather is in flight

    def out_buffer(self):
        return self.bufs[self.k % 2]

    def _finish(self, work, slot):
        work.wait()
        if self.rank == 0:
            self.untile(self.big[slot], slot)

    def submit(self):
        slot = self.k % 2
        self.k += 1
        if self.pending is not None:
            self._finish(*self.pending)
            self.pending = None
        if self.world == 1:
            return
        if self.host_staging:
            import torch
            host = self.bufs[slot].cpu()
            hp = [torch.empty_like(host) for _ in range(self.world)] if self.rank == 0 else None
            self.dist.gather(host, hp, dst=0)
            if self.rank == 0:
                for dst, src in zip(self.parts[slot], hp):
                    dst.copy_(src)
                self.untile(self.big[slot], slot)
            return
        work = self.dist.gather(self.bufs[slot], self.parts[slot] if self.rank == 0 else None, dst=0,
                                async_op=True)
        if self.overlap:
            self.pending = (work, slot)
        else:
            self._finish(work, slot)

    def drain(self):
        if self.pending is not None:
            self._finish(*self.pending)
            self.pending = None


def gather_to_root(local, world, rank, dist):
    """torch.distributed.gather of equally sized tile buffers to rank 0; returns the concatenation on rank 0."""
    import torch
    if world == 1:
        return local
    bufs = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local, bufs, dst=0)
    return torch.cat(bufs) if rank == 0 else None


def mgpu_unique_id():
    """vhx_mgpu_unique_id: rank 0's RCCL communicator id (128 bytes) to send to every rank out of band."""
    buf = (ctypes.c_uint8 * N.VHX_MGPU_ID_BYTES)()
    N.check(N.lib().vhx_mgpu_unique_id(buf))
    return bytes(buf)


class MgpuRenderer:
    """The multi-GPU split behind the C ABI (vhx_mgpu_*): one libvhx context per process and GPU, an RCCL
    communicator owned by libvhx, the tree broadcast from rank 0 over RCCL, and per frame the rank's tiles traced,
    sent to rank 0 over RCCL (RGBA8 + f32 depth) and untiled there. `uid` = the bytes of mgpu_unique_id() created on
    rank 0 (exchange them with e.g. torch.distributed.broadcast_object_list over gloo)."""

    def __init__(self, raytracer, uid, world, rank, tile_size=64, overlap=True):
        self.rt, self.world, self.rank, self.T = raytracer, world, rank, tile_size
        idbuf = (ctypes.c_uint8 * N.VHX_MGPU_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        raytracer._check(N.lib().vhx_mgpu_create(raytracer._h, idbuf, world, rank, tile_size, ctypes.byref(h)))
        self._h = h
        self.set_overlap(overlap)

    def _check(self, rc):
        return self.rt._check(rc)

    def set_overlap(self, on):
        self._check(N.lib().vhx_mgpu_set_overlap(self._h, 1 if on else 0))

    def set_frames_in_flight(self, frames):
        self._check(N.lib().vhx_mgpu_set_frames_in_flight(self._h, frames))

    def broadcast_tree(self, flat=None):
        """Rank 0 passes the FlatTree, the other ranks None (collective)."""
        desc = ctypes.byref(flat.desc) if flat is not None else None
        self._check(N.lib().vhx_mgpu_broadcast_tree(self._h, desc))
        self.rt._tree = flat

    def render(self, cam, fb_rgba=None, fb_depth=None):
        """Collective; rank 0 passes device framebuffers (torch tensors of width*height int32 / float32)."""
        p = lambda t: ctypes.c_void_p(None if t is None else t.data_ptr())
        self._check(N.lib().vhx_mgpu_render(self._h, ctypes.byref(cam), p(fb_rgba), p(fb_depth)))

    def render_batch(self, cams, fb_rgba=None, fb_depth=None):
        """Collective (vhx_mgpu_render_batch): the frames of `cams` as one batch; rank 0 passes lists of device
        framebuffers (one per camera; fb_depth may be None), the other ranks None."""
        n = len(cams)
        cs = (N.Camera * n)(*cams)
        arr = lambda ts: None if ts is None else ctypes.cast((ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]),
                                                             ctypes.c_void_p)
        self._check(N.lib().vhx_mgpu_render_batch(self._h, ctypes.cast(cs, ctypes.c_void_p), n, arr(fb_rgba),
                                                  arr(fb_depth)))

    def sync(self):
        ms = ctypes.c_float()
        self._check(N.lib().vhx_mgpu_sync(self._h, ctypes.byref(ms)))
        return ms.value

    def set_root_slots(self, slots):
        """Collective: rank 0 traces `slots` of the slots + N - 1 tile slots (vhx_mgpu_set_root_slots)."""
        self._check(N.lib().vhx_mgpu_set_root_slots(self._h, slots))

    def set_planes(self, planes):
        """Planes every rank sends to rank 0 (vhx_mgpu_set_planes): 2 = RGBA8 + depth, 1 = RGBA8 only (rank 0 then
        renders with fb_depth=None). Collective: every rank calls it; the ranks agree on the value over the
        communicator, and if they passed different values every rank raises and keeps its previous count."""
        self._check(N.lib().vhx_mgpu_set_planes(self._h, planes))

    def frame_bytes(self, width, height):
        """Bytes rank 0 receives over xGMI per frame at the current split and plane count (vhx_mgpu_frame_bytes)."""
        b = ctypes.c_uint64()
        self._check(N.lib().vhx_mgpu_frame_bytes(self._h, width, height, ctypes.byref(b)))
        return b.value

    def balance(self, cam, frames=4):
        """Collective: measures rank 0's trace and the transfers into it and picks rank 0's share
        (vhx_mgpu_balance); returns (root_slots, trace_ms, transfer_ms)."""
        r, a, g = ctypes.c_uint32(), ctypes.c_float(), ctypes.c_float()
        self._check(N.lib().vhx_mgpu_balance(self._h, ctypes.byref(cam), frames, ctypes.byref(r), ctypes.byref(a),
                                             ctypes.byref(g)))
        return r.value, a.value, g.value

    def measure(self, cam, frames=4):
        """Collective: this rank's median trace and transfer device times (ms) at the current split, frames rendered
        one at a time (vhx_mgpu_measure)."""
        a, g = ctypes.c_float(), ctypes.c_float()
        self._check(N.lib().vhx_mgpu_measure(self._h, ctypes.byref(cam), frames, ctypes.byref(a), ctypes.byref(g)))
        return a.value, g.value

    def rays(self, width, height):
        n = ctypes.c_uint64()
        self._check(N.lib().vhx_mgpu_info(self._h, width, height, None, None, ctypes.byref(n)))
        return n.value

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            N.lib().vhx_mgpu_destroy(self._h)
            self._h = None
