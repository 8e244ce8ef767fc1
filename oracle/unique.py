"""Tuple uniqueness / dedup rank — exact integer restatement. Test infrastructure only.

References:
  * p_unique_ids: modules/rqvae.py:152-157 — (~triu(eq_all, 1)).all(1).sum() / B, i.e. the
    number of rows that have no identical EARLIER row... restated below as the count of
    distinct tuples (identical result: each distinct tuple has exactly one first row).
  * corpus dedup column: modules/tokenizer/semids.py:74-101 — for each item, the number of
    EARLIER items (in corpus order) with an identical L-tuple.
"""
import numpy as np


def count_unique_rows(ids):
    return int(np.unique(np.asarray(ids), axis=0).shape[0])


def dedup_rank(ids):
    """rank[i] = #{j < i : ids[j] == ids[i]} (semids.py:86-94)."""
    ids = np.asarray(ids)
    seen = {}
    out = np.zeros(ids.shape[0], np.int64)
    for i, row in enumerate(map(tuple, ids)):
        out[i] = seen.get(row, 0)
        seen[row] = out[i] + 1
    return out
