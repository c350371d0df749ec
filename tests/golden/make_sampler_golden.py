"""Fixture generator: runs the REFERENCE's ContrastiveBatchSampler (src/datasets/samplers.py) in
the build container and records its batches.  The reference package's src/datasets/__init__.py
imports torchaudio (absent), so samplers.py is loaded on its own by file path; its only import
outside numpy/torch is src.utils.logging, which imports fine.

    PYTHONPATH=/root/reference python tests/golden/make_sampler_golden.py
"""
import importlib.util
import os
import sys

import numpy as np

REF = os.environ.get("PCX_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
spec = importlib.util.spec_from_file_location("src.datasets.samplers", os.path.join(REF, "src/datasets/samplers.py"),
                                              submodule_search_locations=None)
mod = importlib.util.module_from_spec(spec)
mod.__package__ = "src.datasets"
spec.loader.exec_module(mod)

CASES = {
    # name: (labels, classes_per_batch, samples_per_class, views, shuffle, seed, min_exclude)
    "balanced": ([i % 12 for i in range(96)], 6, 2, 2, True, 42, 0),
    "ragged": ([0] * 9 + [1] * 1 + [2] * 4 + [3] * 2 + [4] * 7 + [5] * 3 + [6] * 1 + [7] * 5, 3, 2, 2, True, 7, 0),
    "exclude": ([0] * 9 + [1] * 1 + [2] * 4 + [3] * 2 + [4] * 7 + [5] * 3, 2, 3, 2, True, 3, 3),
    "noshuffle": ([i % 5 for i in range(40)], 2, 4, 2, False, 1, 0),
}

out = {}
for name, (labels, k, m, v, sh, seed, mn) in CASES.items():
    s = mod.ContrastiveBatchSampler(labels, k, m, v, shuffle=sh, seed=seed, min_samples_to_exclude=mn)
    batches = []
    for epoch in range(3):  # the RandomState carries over between epochs
        for b in s:
            batches.append([epoch] + [int(i) for i in b])
    out[name + "/labels"] = np.array(labels, dtype=np.int64)
    out[name + "/cfg"] = np.array([k, m, v, int(sh), seed, mn], dtype=np.int64)
    out[name + "/batches"] = np.array(batches, dtype=np.int64).reshape(len(batches), -1) if batches else \
        np.zeros((0, 1 + k * m), dtype=np.int64)
    out[name + "/len"] = np.array(len(s), dtype=np.int64)
np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "sampler.npz"), **out)
print({k: v.shape for k, v in out.items()})
