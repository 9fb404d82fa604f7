"""ORACLE — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker (or, for
bench, the timed CPU baseline) — never as the thing measured or shipped.  The
product path (``leak-det-gnn_amd/models``) never imports it and has no CPU
fallback.

Modules (each function cites the reference file:line it restates):
  graph_ref     .inp parsing, WDN graph build, batchify, gcn_norm CSR, incidence
                (integer work; restates reference models/utils.py:18-166 and
                 detector.py:105-114; PyG gcn_norm for the CSR)
  gcn_ref       PyG GCNConv / global_mean_pool restated with scatter semantics
  dense_ref     an INDEPENDENT dense formulation of the same two operators
                (Ahat as a dense matrix, pooling as a one-hot matmul)
  detector_ref  LeakDetector forward restated on torch CPU over gcn_ref
  make_golden   fixture generator (imports the reference from /root/reference;
                container-side only)

Pinning:
  * graph builder, batchify, predictor, residual builder: pinned bit-exact /
    to fp32 against fixtures produced by running the reference's own code
    (models/utils.py, models/predictor.py import cleanly here).
  * LeakDetector: pinned against fixtures from the reference detector.py run
    with the INDEPENDENT dense_ref operators supplied as ``torch_geometric.nn``
    (PyG is not installed and is unpinned in the reference), so the
    module structure, ordering and every non-PyG op come from the reference
    itself.  The PyG arithmetic (gcn_norm / propagate / mean pool) is
    "parity unpinned" against PyG proper; it is anchored by two independent
    formulations (scatter gcn_ref vs dense dense_ref) plus a hand-computed
    4-node graph (tests/test_oracle.py).
"""
