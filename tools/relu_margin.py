"""Distance of the flagship's relu inputs from the kink, per graph size (GPU diagnostic).

The aggregate-first GATConv ("xagg", gat_xagg.hip) and the h-first one round differently in fp32
(~1e-7 relative).  An activation whose relu input lies closer to 0 than that can take the other
side of relu' in the two forms, and the gradient of that one element then differs by its whole
value -- a discontinuity of the reference's own arithmetic, not a kernel fault.  At the first
step LayerNorm's beta is 0, so a flipped LN output sits at xhat ~ 0: dgamma is untouched and
dbeta / the block's dW take the jump (the signature seen at n = 777).

    python tools/relu_margin.py 700 777 760 ...   (prints one JSON line per n)

For each n: a world-1 "xagg" forward (SimComm: the collectives of one rank are identities), then
in float64 from that forward's tail input: min |y0| of the GATConv output before its relu and
min |z| of the three LayerNorm outputs before theirs (models.py:637-655).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "hic-gnn_amd"),
           os.path.join(os.path.dirname(HERE), "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def main(ns):
    from test_gpu_dist import xagg_margins     # tail_margins: the float64 LN pre-activations
    for n in ns:
        y0, ln = xagg_margins(n)
        print(json.dumps({"n": n, "gat_y0_min_abs": y0, "ln_min_abs": ln}), flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [300, 777])
