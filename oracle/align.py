"""CPU restatement of the reference's cross-resolution embedding alignment (TEST INFRASTRUCTURE ONLY).

Reference: ``utils.py:83-109`` ``domain_alignment`` (orthogonal Procrustes between the embeddings of
two resolutions of one chromosome), called by ``HiC_GAT_generalize_directly.py:316`` before the
trained model is applied to the untrained resolution.

``scipy.linalg.orthogonal_procrustes(A, B)`` (the reference's dependency, present in this image)
returns R = U V^T from the SVD of A^T B.  When A^T B is rank deficient (fewer matched bins than
embedding dimensions -- the 1 mb -> 500 kb case: ~116 rows against 512 columns) R is not unique in
the null space and depends on the LAPACK build; the optimum ||A R - B||_F and R on the range are.
"""
import numpy as np
from scipy.linalg import orthogonal_procrustes


def matched_rows(list1, list2):
    """Row indices (into embeddings2, embeddings1) of the bins that line up (utils.py:84-104)."""
    idx1 = np.unique(list1[:, 0]).astype(int)
    diff1 = min(idx1[1:] - idx1[:-1])
    idx2 = np.unique(list2[:, 0]).astype(int)
    diff2 = min(idx2[1:] - idx2[:-1])
    bins = (diff1 / (2 * diff2)).astype(int)
    a_rows, b_rows = [], []
    for i in range(bins + 1):
        a_rows.append(np.where(np.isin(idx2 + i * diff2, idx1))[0])
        b_rows.append(np.where(np.isin(idx1, idx2 + i * diff2))[0])
    return np.concatenate(a_rows), np.concatenate(b_rows)


def domain_alignment(list1, list2, embeddings1, embeddings2):
    """utils.py:83-109: embeddings2 rotated onto embeddings1's frame (float64 like numpy)."""
    ia, ib = matched_rows(list1, list2)
    A = embeddings2[ia, :]
    B = embeddings1[ib, :]
    transform = orthogonal_procrustes(A, B)[0]
    return np.matmul(embeddings2, transform), transform, A, B
