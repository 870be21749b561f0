"""Tree writes ordered against frames in flight inside libvhx: writes go through
the owner context (vhx_update_ranges, vhx_upload_tree through a stream resize), frames are traced on eight contexts
sharing the tree, each on its own stream, and nothing is synchronised by the caller in between. Every frame must equal
the oracle on the version of the tree it was submitted against: all writes submitted before it, none after it.
"""
import ctypes

import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests.test_streaming import _edit, _tree

pytestmark = pytest.mark.gpu

F = 8


def _frame_out(n, dev):
    import torch
    return {"rgba": torch.zeros(n, dtype=torch.int32, device=dev),
            "depth": torch.zeros(n, dtype=torch.float32, device=dev),
            "value": torch.zeros(n, dtype=torch.int32, device=dev)}


def _host(o):
    return {k: v.cpu().numpy().view(np.uint32) for k, v in o.items()}


def _same(got, ref, what):
    for k in ("value", "rgba", "depth"):
        r = ref[k].view(np.uint32)
        assert np.array_equal(got[k], r), f"{what}: {k} differs at {(got[k] != r).sum()} pixels"


def _contexts(owner):
    import torch
    ctxs = [owner] + [owner.shared() for _ in range(F - 1)]
    streams = [torch.cuda.ExternalStream(r.stream(), device=torch.device("cuda", 0)) for r in ctxs]
    return ctxs, streams


def test_ranged_writes_between_frames_in_flight(oracle):
    """Three rounds: every context submits a frame of tree version v, the owner writes edit v (voxels cleared, a
    palette write that rebuilds every bitmap, child entries cut), every context submits a frame again. Each first frame
    must show version v (the write waited for it), each second frame version v + 1 (it waited for the write)."""
    import torch
    size, bd, W, H = 256, 4, 320, 200
    build = lambda: vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, bd)  # noqa: E731
    base = build()
    n3 = bd ** 3
    nb = int(base.desc.brick_count)
    pal = base.color_palette.copy()
    pal[1::3] = (pal[1::3] & 0x00FFFFFF) | 0x80000000  # a third of the colours change alpha (still opaque) ...
    pal[2::5] &= 0x00FFFFFF                              # ... and a fifth become fully transparent: empty cells
    root_children = base.node_children[:64].copy()
    root_children[::3] = N.VHX_EMPTY  # every third child entry of the root is cut (occupied, absent: a miss)
    edits = [[(N.VHX_BUF_VOXELS, 0, np.full((nb // 3) * n3, N.VHX_EMPTY, np.uint32))],
             [(N.VHX_BUF_COLOR_PALETTE, 0, pal)],
             [(N.VHX_BUF_NODE_CHILDREN, 0, root_children),
              (N.VHX_BUF_VOXELS, (nb // 2) * n3, np.full(n3 * 64, N.VHX_EMPTY, np.uint32))]]
    versions = [base]
    for k in range(len(edits)):
        v = build()
        for e in edits[:k + 1]:
            for bid, off, vals in e:
                arr = {N.VHX_BUF_VOXELS: v.voxels, N.VHX_BUF_COLOR_PALETTE: v.color_palette,
                       N.VHX_BUF_NODE_CHILDREN: v.node_children}[bid]
                arr[off:off + vals.size] = vals
        versions.append(v)
    cams = [vhx.glass_camera(size, W, H, angle=40.0 + 0.07 * i, target=(size / 2,) * 3) for i in range(F)]
    refs = [[oracle.trace_primary(v, c, 0, 0, W, H, fields=("value", "rgba", "depth")) for c in cams]
            for v in versions]
    for i in range(F):  # the edits are visible in every view
        assert not np.array_equal(refs[0][i]["value"], refs[1][i]["value"])
        assert not np.array_equal(refs[1][i]["rgba"], refs[2][i]["rgba"])
        assert not np.array_equal(refs[2][i]["value"], refs[3][i]["value"])
    owner = vhx.Raytracer(0)
    try:
        owner.upload(base)
        ctxs, streams = _contexts(owner)
        dev = torch.device("cuda", 0)
        before = [[_frame_out(W * H, dev) for _ in range(F)] for _ in edits]
        after = [[_frame_out(W * H, dev) for _ in range(F)] for _ in edits]
        torch.cuda.synchronize()  # the zero fills (torch's stream) complete before the context streams write
        for v, e in enumerate(edits):
            for r, c, o in zip(ctxs, cams, before[v]):
                r.trace_primary(c, out=o)
            owner.update_ranges(e)  # ordered after the frames above, before the frames below
            for r, c, o in zip(ctxs, cams, after[v]):
                r.trace_primary(c, out=o)
        torch.cuda.synchronize()
        for v in range(len(edits)):
            for i in range(F):
                _same(_host(before[v][i]), refs[v][i], f"round {v} context {i}, submitted before the write")
                _same(_host(after[v][i]), refs[v + 1][i], f"round {v} context {i}, submitted after the write")
        for r in ctxs[1:]:
            r.close()
    finally:
        owner.close()


class _Snapshot:
    """A copy of a streamed view's host mirror (the tree version a frame was submitted against)."""

    def __init__(self, view):
        d = view.desc
        n3 = d.brick_dim ** 3
        spec = [("node_type", d.node_count, np.uint32), ("node_ocbits", d.node_count, np.uint64),
                ("node_children", d.node_count * 64, np.uint32), ("voxels", d.brick_count * n3, np.uint32),
                ("solid_values", d.solid_count, np.uint32), ("color_palette", d.color_count, np.uint32),
                ("data_palette", d.data_count, np.uint32)]
        self.desc = N.TreeDesc()
        for f in ("boxtree_size", "brick_dim", "node_count", "brick_count", "solid_count", "color_count", "data_count"):
            setattr(self.desc, f, getattr(d, f))
        self._keep = []
        for name, n, dt in spec:
            ptr = getattr(d, name)
            a = np.zeros(max(1, n), dt)
            if n and ptr:
                a[:n] = np.ctypeslib.as_array((ctypes.c_uint8 * (n * np.dtype(dt).itemsize)).from_address(ptr)).view(dt)
            self._keep.append(a)
            setattr(self.desc, name, a.ctypes.data if n else None)


@pytest.mark.parametrize("batch", [1, 4])
def test_streaming_with_eight_frames_in_flight(oracle, batch):
    """The reference's renderer loop (upload::<T> then dispatch every frame, streaming/mod.rs:420-635,
    pipeline/mod.rs:96-155) with eight frames in flight: per frame the stream's ranged writes (and, when the view
    outgrows its buffers, a re-upload) go through the owner, then the frame is submitted on context k % 8; the viewport
    moves and the tree is edited mid-stream. Every frame equals the oracle on the host mirror as of its submission.
    batch = 4: the uploads of four frames are written once every four frames (vhx_stream_upload_frames), so four frames
    in flight share one tree version."""
    import torch
    size, bd, W, H = 64, 4, 256, 160
    t = _tree(size, bd)
    S = float(size)
    owner = vhx.Raytracer(0)
    try:
        # a small first view that outgrows its device buffers several times (frames 12, 16, 28 of this sequence)
        s = vhx.StreamingView(t, owner, (S / 2, S / 2, S / 2), S / 4)
        s.set_rates(8, 32, 10)
        _, grow = s.upload()
        if grow:
            s.resize()
        ctxs, streams = _contexts(owner)
        dev = torch.device("cuda", 0)
        rng = np.random.default_rng(3)
        frames, snaps, cams, resizes = 40, [], [], 0
        outs = [_frame_out(W * H, dev) for _ in range(frames)]
        torch.cuda.synchronize()  # the zero fills (torch's stream) complete before the context streams write
        for k in range(frames):
            if k in (12, 26):
                _edit(t, rng, size)
            if k == 20:
                s.set_viewport((0.6 * S, 0.5 * S, 0.5 * S), S)
            grow = False
            if k % batch == 0:
                _, grow = s.upload(frames=batch)  # ranged writes through the owner, no host wait
            if grow:
                s.resize()  # re-upload of a larger device view: waits for the frames in flight
                resizes += 1
            snaps.append(_Snapshot(s.view()))
            cam = vhx.glass_camera(size, W, H, angle=40.0 + 0.03 * k, target=(S / 2,) * 3)
            cams.append(cam)
            ctxs[k % F].trace_primary(cam, out=outs[k])
        assert resizes >= (2 if batch == 1 else 1)
        torch.cuda.synchronize()
        changed = 0
        for k in range(frames):
            ref = oracle.trace_primary(snaps[k], cams[k], 0, 0, W, H, fields=("value", "rgba", "depth"))
            _same(_host(outs[k]), ref, f"frame {k} on context {k % F}")
            if k and not np.array_equal(ref["value"], prev):
                changed += 1
            prev = ref["value"]
        assert changed > frames // (2 * batch), "the streamed view should change from upload to upload"
        for r in ctxs[1:]:
            r.close()
        s.close()
    finally:
        owner.close()


def test_upload_tree_device_matches_host_upload(oracle):
    """vhx_upload_tree_device (the receive half of vhx_mgpu_broadcast_tree: counts -> allocation -> device-side fill
    -> derived layout) fed from device tensors: the context traces exactly like the oracle; a shared context of it too."""
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    W, H = 320, 200
    cam = vhx.glass_camera(256, W, H, target=(128.0, 128.0, 128.0))
    ref = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value", "rgba", "depth"))
    dev = torch.device("cuda", 0)
    keep = {}
    d = N.TreeDesc()
    for f in ("boxtree_size", "brick_dim", "node_count", "brick_count", "solid_count", "color_count", "data_count"):
        setattr(d, f, getattr(flat.desc, f))
    for name in ("node_type", "node_ocbits", "node_children", "voxels", "solid_values", "color_palette",
                 "data_palette"):
        a = getattr(flat, name)
        if a.size:
            keep[name] = torch.from_numpy(a.view(np.uint8).copy()).to(dev)
            setattr(d, name, keep[name].data_ptr())
    rt = vhx.Raytracer(0)
    try:
        N.check(N.lib().vhx_upload_tree_device(rt._h, ctypes.byref(d)), rt._h)
        rt._tree = flat  # for Raytracer.shared()
        _same({k: v.view(np.uint32) for k, v in rt.trace_primary(cam, fields=("value", "rgba", "depth")).items()},
              ref, "device upload")
        sh = rt.shared()
        _same({k: v.view(np.uint32) for k, v in sh.trace_primary(cam, fields=("value", "rgba", "depth")).items()},
              ref, "shared context of a device upload")
        sh.close()
        bad = N.TreeDesc()
        ctypes.memmove(ctypes.byref(bad), ctypes.byref(d), ctypes.sizeof(d))
        bad.voxels = None
        assert N.lib().vhx_upload_tree_device(rt._h, ctypes.byref(bad)) == N.VHX_E_INVALID_ARG
    finally:
        rt.close()


def _pal_edit(flat):
    pal = flat.color_palette.copy()
    pal[1::3] = (pal[1::3] & 0x00FFFFFF) | 0x80000000
    pal[2::5] &= 0x00FFFFFF  # transparent: their cells become empty (every bitmap is rebuilt)
    return pal


def test_write_waits_for_a_frame_whose_context_changed_stream(oracle):
    """a shared context traces on its own stream, then is moved onto the owner's stream
    (vhx_set_stream) before the owner writes. The write must still wait for that frame (recorded on the old stream):
    the frame shows the tree before the write, the next frame after it."""
    import torch
    size, W, H = 256, 1920, 1080
    base = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    edited = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    pal = _pal_edit(base)
    edited.color_palette[:] = pal
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    ref0 = oracle.trace_primary(base, cam, 0, 0, W, H, fields=("value", "rgba", "depth"))
    ref1 = oracle.trace_primary(edited, cam, 0, 0, W, H, fields=("value", "rgba", "depth"))
    owner = vhx.Raytracer(0)
    try:
        owner.upload(base)
        sh = owner.shared()
        sh.stream()  # its own stream
        dev = torch.device("cuda", 0)
        o0, o1 = _frame_out(W * H, dev), _frame_out(W * H, dev)
        torch.cuda.synchronize()
        for rep in range(3):
            sh.set_stream(None)
            sh.trace_primary(cam, out=o0)            # on the shared context's own stream
            sh.set_stream(owner.stream())            # moved onto the owner's stream before the write
            owner.update_ranges([(N.VHX_BUF_COLOR_PALETTE, 0, pal if rep % 2 == 0 else base.color_palette)])
            sh.trace_primary(cam, out=o1)            # after the write, on the owner's stream
            torch.cuda.synchronize()
            before, after = (ref0, ref1) if rep % 2 == 0 else (ref1, ref0)
            _same(_host(o0), before, f"rep {rep}: frame submitted before the write")
            _same(_host(o1), after, f"rep {rep}: frame submitted after the write")
        sh.close()
    finally:
        owner.close()


def test_writes_and_traces_from_two_threads(oracle):
    """contexts of one tree driven from two host threads -- one thread traces frames on a shared
    context, the other writes the palette through the owner, alternately. Every frame must show one whole tree version
    (the one before or the one after a write), never a mix: libvhx holds a write until no trace is being submitted and
    a trace until no write is."""
    import threading

    import torch
    size, W, H = 256, 640, 400
    base = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    edited = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    pal = _pal_edit(base)
    edited.color_palette[:] = pal
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    refs = [oracle.trace_primary(f, cam, 0, 0, W, H, fields=("value", "rgba", "depth")) for f in (base, edited)]
    owner = vhx.Raytracer(0)
    try:
        owner.upload(base)
        sh = owner.shared()
        dev = torch.device("cuda", 0)
        outs = [_frame_out(W * H, dev) for _ in range(24)]
        torch.cuda.synchronize()
        errors = []

        def writer():
            try:
                for k in range(24):
                    owner.update_ranges([(N.VHX_BUF_COLOR_PALETTE, 0, pal if k % 2 == 0 else base.color_palette)])
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        th = threading.Thread(target=writer)
        th.start()
        for o in outs:
            sh.trace_primary(cam, out=o)
        th.join()
        assert not errors, errors
        torch.cuda.synchronize()
        seen = set()
        for k, o in enumerate(outs):
            h = _host(o)
            ok = [v for v, r in enumerate(refs) if all(np.array_equal(h[f], r[f].view(np.uint32))
                                                        for f in ("value", "rgba", "depth"))]
            assert ok, f"frame {k} shows neither tree version (a torn read)"
            seen.add(ok[0])
        sh.close()
    finally:
        owner.close()


@pytest.mark.gpu
def test_write_is_not_starved_by_continuous_traces():
    """ADVICE r04 (writer priority): two host threads submit frames back to back on two shared contexts, so the tree
    is almost never free of traces in flight; a third thread's ranged writes must still get in while they run
    (write_begin raises writers_waiting, and trace_begin waits while it is non-zero), not only after they stop."""
    import threading
    import time

    import torch
    size, W, H = 256, 320, 200
    base = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    pal = _pal_edit(base)
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    owner = vhx.Raytracer(0)
    try:
        owner.upload(base)
        tracers = [owner.shared(), owner.shared()]
        dev = torch.device("cuda", 0)
        outs = [_frame_out(W * H, dev) for _ in tracers]
        torch.cuda.synchronize()
        stop, errors, frames, write_done = threading.Event(), [], [0, 0], []

        def trace(i):
            try:
                while not stop.is_set() and frames[i] < 200000:
                    tracers[i].trace_primary(cam, out=outs[i])
                    frames[i] += 1
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        ths = [threading.Thread(target=trace, args=(i,)) for i in range(2)]
        for th in ths:
            th.start()
        tw = time.perf_counter()
        while min(frames) < 20 and not errors and time.perf_counter() - tw < 60:  # both tracers running
            time.sleep(0.001)
        t0 = time.perf_counter()
        for k in range(6):
            owner.update_ranges([(N.VHX_BUF_COLOR_PALETTE, 0, pal if k % 2 == 0 else base.color_palette)])
        write_done.append(time.perf_counter() - t0)
        running = [th.is_alive() for th in ths]
        stop.set()
        for th in ths:
            th.join(timeout=120)
        assert not errors, errors
        assert all(running), "the tracers stopped before the writes completed: the writes were starved"
        assert write_done[0] < 30.0, write_done
        torch.cuda.synchronize()
        for t in tracers:
            t.close()
    finally:
        owner.close()


@pytest.mark.gpu
def test_depth_prepass_frames_with_concurrent_writes():
    """a depth-prepass frame traces its half-resolution frame from inside its own trace scope. With
    writer priority, a write queued between the outer and the inner trace_begin used to wait for the outer trace while
    the inner one waited for the writer: both threads blocked for good. The inner frame now joins the outer scope;
    prepass frames on two shared contexts and ranged writes from a third thread must all complete."""
    import threading
    import time

    import torch
    size, W, H = 256, 320, 200
    base = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    pal = _pal_edit(base)
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    owner = vhx.Raytracer(0)
    try:
        owner.upload(base)
        tracers = [owner.shared(), owner.shared()]
        for t in tracers:
            t.set_depth_prepass(True, 0.5)
        dev = torch.device("cuda", 0)
        outs = [_frame_out(W * H, dev) for _ in tracers]
        torch.cuda.synchronize()
        stop, errors, frames = threading.Event(), [], [0, 0]

        def trace(i):
            try:
                while not stop.is_set() and frames[i] < 100000:
                    tracers[i].trace_primary(cam, out=outs[i])
                    frames[i] += 1
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        ths = [threading.Thread(target=trace, args=(i,), daemon=True) for i in range(2)]
        for th in ths:
            th.start()
        tw = time.perf_counter()
        while min(frames) < 10 and not errors and time.perf_counter() - tw < 60:
            time.sleep(0.001)
        done = []

        def writer():
            for k in range(40):
                owner.update_ranges([(N.VHX_BUF_COLOR_PALETTE, 0, pal if k % 2 == 0 else base.color_palette)])
            done.append(True)

        wt = threading.Thread(target=writer, daemon=True)
        wt.start()
        wt.join(timeout=60)
        stop.set()
        for th in ths:
            th.join(timeout=60)
        assert not errors, errors
        assert done, "the writes did not complete: deadlock between a prepass frame and a writer"
        assert not any(th.is_alive() for th in ths), "a prepass tracer never returned: deadlock"
        torch.cuda.synchronize()
        for t in tracers:
            t.close()
    finally:
        owner.close()
