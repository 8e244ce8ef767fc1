"""Lloyd k-means used for codebook init — numpy restatement. Test infrastructure only.

Reference: init/kmeans.py:23-74. Init = x[np.random.choice(B, k, replace=False)] (:34-38);
each iteration assigns by argmin of the broadcast squared difference sum (:40-44), then
every centroid becomes the mean of its members (empty clusters get a random row, :49-55);
stops when max centroid move < stop_threshold (:67-68) or after max_iters.
"""
import numpy as np


def kmeans(x, init_idx, max_iters, stop_threshold=1e-10):
    x = x.astype(np.float32)
    c = x[init_idx].copy()
    assign = None
    for _ in range(max_iters):
        old = c.copy()
        d = ((x[:, None, :] - c[None, :, :]) ** 2).sum(2)
        assign = d.argmin(1)
        for j in range(c.shape[0]):
            m = assign == j
            if m.any():
                c[j] = x[m].mean(0)
            else:
                raise NotImplementedError("empty cluster (reference draws a torch.randint row)")
        if np.linalg.norm(c - old, axis=1).max() < stop_threshold:
            break
    return c, assign
