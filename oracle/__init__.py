"""CPU oracle for the phoneme-contrast train step — TEST INFRASTRUCTURE, NOT PRODUCT.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
package, and only as the checker / the timed CPU baseline.  The shipped path
(`phoneme_contrast_amd`) never imports it and fails loudly when its HIP library is missing.

Contents
  np_ops.py     float64 numpy restatement of every op on the path, forward AND hand-written
                backward (no autograd), each citing the reference file:line it restates.
  np_models.py  PhonemeNet / PhonemeNetDeep train step (forward, SupCon, backward, Adam) and
                eval forward on a reference-format state_dict.
  torch_port.py float32 torch-CPU restatement (functional, autograd) used as the timed CPU
                baseline ("kind": "port") and for quick large-batch checks.

Pinning: both restatements are checked against fixtures generated from the reference itself
(`tests/golden/make_golden.py`, run in the build container where the reference is importable);
see tests/test_oracle_golden.py.  Parity is therefore *pinned* (not "unpinned").
"""
