"""CPU oracle — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker (or as
the timed CPU baseline).  The product path (the modules next to libcdr.so)
never imports it: without the HIP library the product fails loudly.

Contents
--------
kmeans_oracle    NumPy restatement of src/kmeans_plusplus.py (bit-exact;
                 pinned against the imported reference: tests/golden/*).
scoring_oracle   np.median + the category scorer of src/scoring.py.
features_oracle  pandas restatement of src/compute_features.py (Spark job).
                 PARITY UNPINNED for Spark-specific timestamp parsing: PySpark
                 and Java are absent here, so no reference run pins it; the
                 integer counts are pinned by construction (independent
                 group-by) and by hand-checked fixtures.
synth            NumPy mirror of the device point generator.
gen_golden       the script that imported the reference to write tests/golden.
"""
