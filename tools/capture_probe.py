"""Probe (GPU box, its own process): what the HIP runtime does with a stream that, inside a graph
capture, waits on an event of a side stream that was ALREADY joined back into the origin -- the
pattern of round 5's slab step (hicgat.streams rule 2) -- against the same steps in the legal order.

  python tools/capture_probe.py ok|rule2

Per trial: the side stream adds 1, the comm stream adds 100 after the side's event; three replays
of a correct graph give 303 and leave 0 after the capture itself (capture executes nothing).
Printed: x after the capture, x after three replays, and whether the comm stream still reports an
active capture after capture_end (a stream left attached to a finished capture).
"""
import sys

import torch


def main():
    pattern = sys.argv[1] if len(sys.argv) > 1 else "ok"
    origin, side, cs = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    for trial in range(4):
        g = torch.cuda.CUDAGraph()
        x.zero_()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=origin):
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                x.add_(1)
            ev = torch.cuda.Event()
            ev.record(side)
            if pattern == "rule2":
                cur.wait_stream(side)          # the lane joined back first ...
            cs.wait_event(ev)                  # ... then another stream waits on its event
            with torch.cuda.stream(cs):
                x.add_(100)
            if pattern != "rule2":
                cur.wait_stream(side)
            cur.wait_stream(cs)
        torch.cuda.synchronize()
        after_capture = float(x.item())
        with torch.cuda.stream(cs):
            cs_capturing = torch.cuda.is_current_stream_capturing()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        print(f"{pattern} trial {trial}: after capture {after_capture:g}, after 3 replays {float(x.item()):g} "
              f"(expected 0 / 303), comm stream still capturing: {cs_capturing}", flush=True)
        del g


if __name__ == "__main__":
    main()
