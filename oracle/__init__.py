"""CPU oracle for the HiC-GNN / GAT-HiC per-epoch hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (``hic-gnn_amd/hicgat``) imports this
package.  Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``
may import it, and only as the checker / the timed CPU baseline -- never as the thing measured or
shipped.

It is a plain-torch (CPU, fp32/fp64) restatement of the reference algorithm:

* ``oracle.graph``  -- ``utils.convert_to_matrix`` / ``utils.load_input`` / ``utils.cont2dist`` and
  torch_sparse ``to_symmetric`` + ``set_diag`` (reference ``utils.py:10-80``).
* ``oracle.gat``    -- PyG 1.7.2 ``GATConv`` semantics (un-vendored third-party; restated from its
  published algorithm) and the two in-scope model classes
  (``models.py:614-691`` and ``models.py:1010-1047``).
* ``oracle.loop``   -- MSE / combined MSE+Pearson loss, Adam, the ``HiC-GNN_main.py:117-132``
  training loop (fixed-K and threshold-stopped) and dSCC (``HiC-GNN_main.py:135-139``).

Pinning: ``tests/golden/make_golden.py`` imports the reference ``utils.py`` / ``models.py`` in the
build container (with small stubs for the absent torch_geometric / torch_sparse packages) and writes
the fixtures under ``tests/golden/``; ``tests/test_oracle_golden.py`` checks this oracle against
them.  The GATConv arithmetic itself is restated from PyG 1.7.2 and is therefore *parity unpinned*
by the reference (the reference ships no GAT outputs); see DESIGN.md section "Oracle".
"""
