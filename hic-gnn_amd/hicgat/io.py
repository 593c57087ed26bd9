"""On-disk formats of the reference outputs.

``write_pdb`` reproduces utils.WritePDB (utils.py:149-192) byte for byte: a leading blank line,
one ATOM record per bead, CONECT i i+1 for every bead including the last one (ctype "0": the
reference writes ``CONECT N N+1``), and a final "END" without newline.
"""


def write_pdb(positions, pdb_file, ctype="0"):
    n = len(positions)
    lines = ["\n"]
    for i in range(1, n + 1):
        p = positions[i - 1]
        c2 = str(i).rjust(5)
        c4 = ("B" + str(i)).ljust(6)
        xs = [("%.3f" % p[k]).rjust(8) for k in range(3)]
        lines.append("%s  %s   %s %s   %s%s%s  %s\n" % ("ATOM", c2, "CA MET", c4, xs[0], xs[1], xs[2], "0.20 10.00"))
    for i in range(1, n + 1):
        j = i + 1
        if j > n and ctype == "1":
            continue
        lines.append("CONECT%s%s\n" % (str(i).rjust(5), str(j).rjust(5)))
    lines.append("END")
    with open(pdb_file, "w") as fh:
        fh.write("".join(lines))


def read_pdb_coords(pdb_file):
    import numpy as np
    xyz = []
    with open(pdb_file) as fh:
        for line in fh:
            if line.startswith("ATOM"):
                xyz.append([float(line[30:38]), float(line[38:46]), float(line[46:54])])
    return np.array(xyz)
