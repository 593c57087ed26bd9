"""hicgat.streams' capture ledger on stand-in streams / events (no GPU): the four rules that keep a
captured step's cross-stream dependencies inside what the HIP runtime's capture supports, and the
fork / join pattern the sharded slab step now follows ("Streams and capture")."""
import pytest
import torch

from hicgat import streams


class FakeStream:
    def __init__(self, h):
        self.cuda_stream = h
        self.waited = []

    def wait_event(self, ev):
        self.waited.append(ev.s.cuda_stream)

    def wait_stream(self, s):
        self.waited.append(s.cuda_stream)


class FakeEvent:
    def record(self, s):
        self.s = s


@pytest.fixture()
def fakes(monkeypatch):
    monkeypatch.setattr(torch.cuda, "Event", FakeEvent)
    yield FakeStream(1), FakeStream(2), FakeStream(3), FakeStream(4)
    streams.LEDGER.active = False


def test_fork_record_wait_join_is_accepted(fakes):
    origin, side, cs, _ = fakes
    streams.begin_capture(origin)
    streams.fork(side, origin)
    ev = streams.record(side)          # the lane's work is done ...
    streams.wait(cs, ev)               # ... the comm stream starts from it while the lane is still forked
    streams.check_launch(cs.cuda_stream)
    streams.join(origin, side)
    streams.join(origin, cs)
    streams.end_capture()
    assert not streams.LEDGER.active
    assert origin.waited == [2, 3] and cs.waited == [2]


def test_wait_on_a_joined_streams_event_is_rejected(fakes):
    """Rule 2 -- the round-5 slab pattern: events recorded on the side lanes, the lanes joined back
    (ops.side_join), THEN the comm stream made to wait on those events."""
    origin, side, cs, _ = fakes
    streams.begin_capture(origin)
    streams.fork(side, origin)
    ev = streams.record(side)
    streams.join(origin, side)
    with pytest.raises(streams.CaptureError, match="rule 2"):
        streams.wait(cs, ev)
    assert cs.waited == []             # rejected before the runtime saw it
    streams.end_capture()              # nothing left open: ends cleanly
    # a re-fork of the lane opens a new epoch: events recorded after it are fine again
    streams.begin_capture(origin)
    streams.fork(side, origin)
    streams.wait(cs, streams.record(side))
    streams.join(origin, side)
    streams.join(origin, cs)
    streams.end_capture()


def test_events_from_outside_the_capture_are_rejected(fakes):
    origin, side, _, _ = fakes
    ev = streams.record(origin)                    # eager (e.g. a warm-up step's event)
    streams.begin_capture(origin)
    with pytest.raises(streams.CaptureError, match="rule 1"):
        streams.wait(side, ev)
    old = streams.record(origin)
    streams.end_capture()
    streams.begin_capture(origin)                  # an event of the PREVIOUS capture
    with pytest.raises(streams.CaptureError, match="rule 1"):
        streams.wait(side, old)
    streams.end_capture()


def test_unjoined_streams_are_joined_then_reported(fakes):
    """Rule 4: the open stream is joined into the origin (so the runtime's capture can end) and the
    capture fails loudly."""
    origin, side, _, stray = fakes
    streams.begin_capture(origin)
    streams.fork(side, origin)
    with pytest.raises(streams.CaptureError, match="rule 3|not part of the capture"):
        streams.check_launch(stray.cuda_stream)
    with pytest.raises(streams.CaptureError, match="not joined back"):
        streams.end_capture()
    assert origin.waited == [2] and not streams.LEDGER.active


def test_outside_a_capture_everything_is_plain(fakes):
    origin, side, cs, _ = fakes
    streams.fork(side, origin)
    ev = streams.record(side)
    streams.join(origin, side)
    streams.wait(cs, ev)               # fine eagerly
    streams.check_launch(99)
    assert cs.waited == [2]
