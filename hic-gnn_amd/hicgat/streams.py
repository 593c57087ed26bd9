"""The step's streams and the capture ledger.

Streams.  ``get(name, device)`` is THE stream of that name on that device: made once, on first use,
by libhicgat (``hicgat_stream_create``: a non-blocking HIP stream) and wrapped as a
``torch.cuda.ExternalStream``; it lives as long as the process.  Names in use: "capture" (the
origin stream of every ``graphs.CapturedStep``), "warm" (its eager warm-up), "side0", "side2",
"side4", "side5", "side6" (``ops``' parameter-gradient lanes), "comm" (the slab / allgather forms'
tail gradient bucket) and "grad" (the xagg form's side branch).  Until round 5 every trainer,
``CapturedStep`` and lane asked torch for a new stream; torch hands out its pool of 32 streams
round robin, so after a few trainers in one process two "different" lanes of a step, or a lane and
the capture stream, could be one HIP stream, and the overlap a step was built for silently
became a serial chain.

Ledger.  Every cross-stream dependency of the step goes through ``record`` / ``wait`` / ``fork`` /
``join`` below.  While a ``CapturedStep`` captures (``begin_capture(origin)`` .. ``end_capture()``), the ledger knows which
streams have joined the capture and enforces:

1. an event waited on inside the capture was recorded inside THIS capture;
2. an event recorded on a side stream is waited on only while that stream is still forked, i.e.
   not yet joined back into the origin since the record (events on the origin are always fine);
3. every library launch (``_lib.stream``, ``check_launch``) is on the origin or a forked stream;
4. when the captured function returns, every forked stream has been joined back into the origin.

A violation raises ``CaptureError``; for rule 4 the open streams are joined first, so the capture
itself still ends cleanly before the error propagates.  Outside a capture the functions are plain
stream operations (events are still tagged, so an event from an eager step cannot be waited on in
a later capture).

Rule 2 is the pattern the round-5 slab step had when its captures aborted (a ``capture_end``
segfault and a core dump, both in the slab form with the simulated communicator; DESIGN.md section
6, "Streams and capture"): it recorded events on the side lanes after their parameter-gradient
launches, joined the lanes back (``ops.side_join``), and only then made the comm stream wait on
those events before its gradient all-reduce.  The bare pattern alone did not fault in a standalone
probe (tools/capture_probe.py); the streams of the same runs also aliased through torch's pool (see
above).  Both are gone, and the ledger keeps the step inside the fork / join forms that are known
to replay.
"""
import ctypes
import threading

import torch


class CaptureError(RuntimeError):
    """A cross-stream dependency inside a graph capture that the HIP runtime does not support."""


_STREAMS = {}
_LOCK = threading.Lock()
NAMES = ("capture", "warm", "side0", "side2", "side4", "side5", "side6", "comm", "grad")


def _dev(device):
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device)
    return torch.device("cuda", torch.cuda.current_device() if d.index is None else d.index)


def get(name, device=None):
    """The process-lifetime stream ``name`` on ``device`` (default: the current device)."""
    if name not in NAMES:
        raise ValueError(f"unknown stream name {name!r} (one of {NAMES})")
    dev = _dev(device)
    key = (dev.index, name)
    s = _STREAMS.get(key)
    if s is None:
        with _LOCK:
            s = _STREAMS.get(key)
            if s is None:
                from . import _lib
                lib = _lib.lib()
                h = ctypes.c_void_p()
                with torch.cuda.device(dev):
                    _lib.check(lib.hicgat_stream_create(0, ctypes.byref(h)), "hicgat_stream_create")
                s = torch.cuda.ExternalStream(h.value, device=dev)
                _STREAMS[key] = s
    return s


def made():
    """{(device index, name): stream handle} of the streams made so far (tests)."""
    return {k: v.cuda_stream for k, v in _STREAMS.items()}


class _Ledger:
    def __init__(self):
        self.active = False
        self.cid = 0
        self.origin = None
        self.open = {}     # handle -> stream, side streams forked into the current capture
        self.epoch = {}    # handle -> number of joins back into the origin during this capture
        self.log = []      # (op, stream handle[, other]) of the current capture, for error messages


LEDGER = _Ledger()


def _h(s):
    return s.cuda_stream


def capturing():
    return LEDGER.active


def begin_capture(origin):
    L = LEDGER
    if L.active:
        raise CaptureError("nested capture")
    L.active, L.cid = True, L.cid + 1
    L.origin = _h(origin)
    L.origin_stream = origin
    L.open, L.epoch, L.log = {}, {}, []


def end_capture():
    """Rule 4: join every still-open stream into the origin (so the capture can end), then raise
    if there was one.  Always leaves the ledger inactive."""
    L = LEDGER
    try:
        left = dict(L.open)
        for h, s in left.items():
            L.origin_stream.wait_stream(s)
        if left:
            raise CaptureError(f"{len(left)} forked stream(s) not joined back into the capture's origin stream "
                               f"before the capture ended: {sorted(hex(h) for h in left)}")
    finally:
        L.active = False
        L.open, L.epoch = {}, {}


def record(stream=None):
    """An event recorded now on ``stream`` (default: the current stream), tagged for the ledger."""
    s = torch.cuda.current_stream() if stream is None else stream
    ev = torch.cuda.Event()
    ev.record(s)
    L = LEDGER
    h = _h(s)
    if L.active:
        if h != L.origin and h not in L.open:
            raise CaptureError(f"event recorded on stream {hex(h)}, which is not part of the capture "
                               f"(fork it from the origin first)")
        ev._hicgat_tag = (L.cid, h, L.epoch.get(h, 0))
    else:
        ev._hicgat_tag = (None, h, None)
    return ev


def wait(stream, ev):
    """``stream`` waits for ``ev`` (an event from ``record``); inside a capture, rules 1-2, and a
    stream that was not yet part of the capture joins it (a fork)."""
    L = LEDGER
    h = _h(stream)
    if L.active:
        tag = getattr(ev, "_hicgat_tag", None)
        if tag is None:
            raise CaptureError("waiting on an event not made by hicgat.streams.record inside a capture")
        cid, eh, ep = tag
        if cid != L.cid:
            raise CaptureError("waiting on an event recorded outside this capture (rule 1)")
        if eh != L.origin and L.epoch.get(eh, 0) != ep:
            raise CaptureError(f"waiting on an event recorded on side stream {hex(eh)} after that stream was "
                               f"joined back into the origin (rule 2): record the event and wait on it before "
                               f"the join")
        if h != L.origin and h not in L.open:
            L.open[h] = stream
        L.log.append(("wait", h, eh))
    stream.wait_event(ev)


def fork(side, src=None):
    """``side`` continues from the current point of ``src`` (default: the current stream)."""
    wait(side, record(src))


def join(dst, side):
    """``dst`` waits for everything issued on ``side`` so far; joining into the capture's origin ends
    ``side``'s part in the capture (its earlier events may no longer be waited on: rule 2)."""
    wait(dst, record(side))
    L = LEDGER
    if L.active and _h(dst) == L.origin:
        h = _h(side)
        if h != L.origin:
            L.epoch[h] = L.epoch.get(h, 0) + 1
            L.open.pop(h, None)
            L.log.append(("join", h))


def check_launch(handle):
    """Rule 3, for every library launch (``_lib.stream``)."""
    L = LEDGER
    if L.active and handle != L.origin and handle not in L.open:
        raise CaptureError(f"library launch on stream {hex(handle)}, which is not part of the capture "
                           f"(neither the origin nor a forked stream)")


# ---- branch stamps (tests/test_gpu_z_overlap.py) --------------------------------------------------
# When ``STAMPS`` is a CUDA uint64 tensor, ``stamp(name)`` enqueues ``hicgat_wall_stamp`` on the
# current stream at the step's fork / join points, so a captured step records, on every replay, the
# device wall clock at which each branch started and ended.  None (the default): no launch at all.
STAMPS = None
SLOTS = {"src_begin": 0, "src_end": 1, "side_begin": 2, "side_end": 3,
         "edge_begin": 4, "edge_end": 5, "grad_begin": 6, "grad_end": 7}


def stamp(name):
    buf = STAMPS
    if buf is None:
        return
    from . import _lib
    _lib.check(_lib.lib().hicgat_wall_stamp(_lib.ptr(buf), SLOTS[name], _lib.stream(buf.device)), "hicgat_wall_stamp")
