"""ctypes binding of libhicgat.so (the C ABI in include/hicgat.h).

The library is built in-tree (``make -C hic-gnn_amd`` or ``__graft_entry__.build()``).  There is
no fallback: if the library or a GPU is missing every op raises ``HicgatUnavailable``.
"""
import ctypes
import os

import torch

from . import streams as _streams

_HERE = os.path.dirname(os.path.abspath(__file__))
# HICGAT_LIB lets tools/kbench.py A/B an alternative build of the same ABI in one process
LIB_PATH = os.environ.get("HICGAT_LIB", os.path.join(_HERE, "libhicgat.so"))

c_int, c_i64, c_f, c_d, c_sz, c_p = (ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double,
                                     ctypes.c_size_t, ctypes.c_void_p)
c_u64 = ctypes.c_uint64


class WgradJob(ctypes.Structure):
    """include/hicgat.h hicgat_wgrad_job."""
    _fields_ = [("dy", c_p), ("ldy", c_i64), ("x", c_p), ("ldx", c_i64), ("dw", c_p), ("lddw", c_i64), ("db", c_p),
                ("M", c_int), ("N", c_int), ("K", c_int), ("accumulate", c_int)]


class ColsumJob(ctypes.Structure):
    """include/hicgat.h hicgat_colsum_job."""
    _fields_ = [("src", c_p), ("ld", c_i64), ("rows", c_i64), ("cols", c_i64), ("dst", c_p), ("accumulate", c_int),
                ("wt", c_p), ("ldw", c_i64), ("segs", c_int), ("ldd", c_i64)]


class GemmJob(ctypes.Structure):
    """include/hicgat.h hicgat_gemm_job."""
    _fields_ = [("a", c_p), ("lda", c_i64), ("b", c_p), ("ldb", c_i64), ("c", c_p), ("ldc", c_i64), ("c_relu", c_p),
                ("ldr", c_i64), ("bias", c_p), ("M", c_int), ("N", c_int), ("K", c_int)]


c_wjobs, c_cjobs, c_gjobs = ctypes.POINTER(WgradJob), ctypes.POINTER(ColsumJob), ctypes.POINTER(GemmJob)

# name -> (restype, argtypes); mirrors include/hicgat.h one to one
SIGNATURES = {
    "hicgat_version": (c_int, []),
    "hicgat_strerror": (ctypes.c_char_p, [c_int]),
    "hicgat_csr_from_dense": (c_int, [c_p, c_int, c_i64, c_p, c_p, c_p, c_sz, c_p]),
    "hicgat_csr_workspace_bytes": (c_sz, [c_int]),
    "hicgat_cont2dist": (c_int, [c_p, c_int, c_i64, c_d, c_p, c_p, c_i64, c_p, c_sz, c_p]),
    "hicgat_cont2dist_workspace_bytes": (c_sz, [c_int]),
    "hicgat_gat_linear_att": (c_int, [c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p]),
    "hicgat_gat_att_logits": (c_int, [c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p]),
    "hicgat_gat_agg_fwd": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p,
                                   c_p, c_f, c_p, c_p, c_p]),
    "hicgat_gat_agg_fwd_act": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p,
                                       c_p, c_f, c_int, c_p, c_p, c_p, c_p]),
    "hicgat_gat_agg_bwd_dst": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p,
                                       c_f, c_p, c_p]),
    "hicgat_gat_agg_bwd_rows": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p,
                                        c_i64, c_p, c_p]),
    "hicgat_gat_agg_bwd_src_ld": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p,
                                          c_i64, c_p, c_i64, c_p, c_p, c_f, c_p, c_p, c_p]),
    "hicgat_gat_agg_bwd_src_ex": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p,
                                          c_i64, c_p, c_i64, c_p, c_p, c_f, c_p, c_p, c_int, c_p]),
    "hicgat_gat_agg_bwd_src": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p,
                                       c_p, c_p, c_p, c_f, c_p, c_p, c_p]),
    "hicgat_gat_agg_fwd_tiled": (c_int, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int,
                                         c_int, c_p, c_p, c_p, c_p, c_f, c_int, c_p, c_p, c_p, c_int, c_p, c_sz,
                                         c_p]),
    "hicgat_gat_agg_bwd_src_tiled": (c_int, [c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                             c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p, c_f, c_p, c_p, c_int,
                                             c_p, c_sz, c_p]),
    "hicgat_gat_tiled_workspace_bytes": (c_sz, [c_int, c_int]),
    "hicgat_gat_param_grad": (c_int, [c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_int, c_p,
                                      c_sz, c_p]),
    "hicgat_gat_param_grad_workspace_bytes": (c_sz, [c_int, c_int]),
    "hicgat_pairdist_fwd": (c_int, [c_p, c_int, c_p, c_i64, c_p]),
    "hicgat_pairdist_bwd": (c_int, [c_p, c_p, c_int, c_i64, c_p, c_p, c_sz, c_p]),
    "hicgat_pairdist_mse_fused": (c_int, [c_p, c_p, c_int, c_i64, c_i64, c_i64, c_int, c_p, c_p, c_p,
                                          c_p, c_sz, c_p]),
    "hicgat_pairdist_mse_fused_band": (c_int, [c_p, c_p, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_int,
                                               c_p, c_p, c_p, c_p, c_sz, c_p]),
    "hicgat_pairdist_finalize": (c_int, [c_int, c_int, c_p, c_p, c_p]),
    "hicgat_pairdist_finalize_rows": (c_int, [c_int, c_int, c_p, c_p, c_p, c_int, c_int, c_p, c_p]),
    "hicgat_pairdist_finalize_rows_ex": (c_int, [c_int, c_int, c_p, c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p, c_p]),
    "hicgat_pairdist_num_tiles": (c_i64, [c_int, c_int]),
    "hicgat_pairdist_workspace_bytes": (c_sz, [c_int, c_int]),
    "hicgat_pairdist_mse_fused_support": (c_int, [c_p, c_int, c_f, c_p, c_p, c_p, c_p, c_int, c_p, c_p, c_p, c_p,
                                                  c_sz, c_p]),
    "hicgat_pairdist_support_workspace_bytes": (c_sz, [c_int]),
    "hicgat_xagg_vec_bytes": (c_sz, []),
    "hicgat_xagg_logits": (c_int, [c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p]),
    "hicgat_xagg_logits_zero": (c_int, [c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_i64,
                                        c_p, c_p]),
    "hicgat_xagg_logits_zero_pack": (c_int, [c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p,
                                             c_i64, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "hicgat_xagg_fwd": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_f, c_p, c_p,
                                c_p]),
    "hicgat_xagg_bias_relu": (c_int, [c_p, c_p, c_p, c_int, c_int, c_p]),
    "hicgat_xagg_rows_bwd": (c_int, [c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p]),
    "hicgat_xagg_edge": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p,
                                 c_f, c_p, c_p]),
    "hicgat_xagg_edge_acc": (c_int, [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p,
                                     c_p, c_f, c_p, c_p]),
    "hicgat_xagg_edge_acc_blocks": (c_int, [c_int]),
    "hicgat_xagg_slab_workspace_bytes": (c_sz, []),
    "hicgat_xagg_slab_sum": (c_int, [c_p, c_p, c_int, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "hicgat_xagg_param_finish": (c_int, [c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_p]),
    "hicgat_xagg_param_finish_seg": (c_int, [c_p, c_p, c_p, c_p, c_p, c_int, c_i64, c_int, c_int, c_int, c_p, c_p,
                                             c_p, c_p]),
    "hicgat_pairdist_mse_fused_support_range": (c_int, [c_p, c_int, c_f, c_p, c_p, c_p, c_p, c_i64, c_i64, c_int,
                                                        c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "hicgat_pairdist_mse_fused_support_range_ex": (c_int, [c_p, c_p, c_int, c_f, c_p, c_p, c_p, c_p, c_i64, c_i64,
                                                           c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "hicgat_truth_support": (c_int, [c_p, c_int, c_i64, c_f, c_p, c_p, c_p, c_p, c_p]),
    "hicgat_gemm": (c_int, [c_int, c_int, c_int, c_int, c_int, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_int,
                            c_int, c_p, c_sz, c_p]),
    "hicgat_gemm_workspace_bytes": (c_sz, [c_int, c_int, c_int]),
    "hicgat_gemm_ex": (c_int, [c_int, c_int, c_int, c_int, c_int, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_int,
                               c_int, c_int, c_p, c_sz, c_p]),
    "hicgat_gemm_wgrad": (c_int, [c_int, c_int, c_int, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_int, c_int, c_p,
                                  c_sz, c_p]),
    "hicgat_gemm_wgrad_workspace_bytes": (c_sz, [c_int, c_int, c_int]),
    "hicgat_gemm_rows_grouped_workspace_bytes": (c_sz, [c_gjobs, c_int, c_int]),
    "hicgat_gemm_rows_grouped": (c_int, [c_gjobs, c_int, c_int, c_int, c_p, c_sz, c_p]),
    "hicgat_param_grads_workspace_bytes": (c_sz, [c_wjobs, c_int, c_int]),
    "hicgat_param_grads_grouped": (c_int, [c_wjobs, c_int, c_cjobs, c_int, c_int, c_p, c_sz, c_p]),
    "hicgat_colsum": (c_int, [c_p, c_i64, c_int, c_int, c_p, c_int, c_p, c_sz, c_p]),
    "hicgat_colsum_workspace_bytes": (c_sz, [c_int, c_int]),
    "hicgat_ln_relu_res_fwd": (c_int, [c_p, c_i64, c_int, c_int, c_p, c_p, c_f, c_p, c_i64, c_p, c_p, c_p]),
    "hicgat_ln_relu_res_bwd": (c_int, [c_p, c_p, c_i64, c_int, c_int, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p,
                                       c_p, c_int, c_p, c_sz, c_p]),
    "hicgat_ln_relu_res_workspace_bytes": (c_sz, [c_int]),
    "hicgat_ln_relu_res_bwd_params": (c_int, [c_int, c_p, c_p, c_int, c_p, c_sz, c_p]),
    "hicgat_tail_pack_bytes": (c_sz, []),
    "hicgat_tail_pack": (c_int, [c_p, c_p, c_p, c_p, c_sz, c_p]),
    "hicgat_tail_fwd_fused": (c_int, [c_p, c_i64, c_int] + [c_p] * 14 + [c_f] + [c_p] * 10 + [c_p, c_p]),
    "hicgat_tail_bwd_waves": (c_int, []),
    "hicgat_tail_bwd_workspace_bytes": (c_sz, [c_int, c_int]),
    "hicgat_tail_bwd_fused": (c_int, [c_p, c_int] + [c_p] * 16 + [c_p] * 4 + [c_p, c_sz] * 3 + [c_p, c_p]),
    "hicgat_tail_fwd_fused_heads": (c_int, [c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_int] + [c_p] * 14 + [c_f]
                                    + [c_p] * 10 + [c_p, c_p]),
    "hicgat_tail_bwd_fused_rows": (c_int, [c_p, c_int] + [c_p] * 16 + [c_p] * 3 + [c_p, c_sz] * 3
                                   + [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "hicgat_tail_bwd_fused_heads": (c_int, [c_p, c_int] + [c_p] * 16 + [c_p] * 3 + [c_p, c_sz] * 3
                                    + [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "hicgat_sage_weights": (c_int, [c_p, c_int, c_i64, c_p, c_p, c_p, c_p, c_p]),
    "hicgat_sage_agg": (c_int, [c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_p, c_int, c_int, c_p, c_i64,
                                c_p]),
    "hicgat_kr_matvec": (c_int, [c_p, c_i64, c_int, c_p, c_p, c_p, c_p, c_p]),
    "hicgat_kr_scale": (c_int, [c_p, c_i64, c_int, c_p, c_p, c_i64, c_p]),
    "hicgat_n2v_walks": (c_int, [c_p, c_p, c_p, c_int, c_p, c_int, c_int, c_f, c_f, c_u64, c_p, c_p]),
    "hicgat_n2v_sgns_epoch": (c_int, [c_p, c_int, c_int, c_p, c_p, c_int, c_int, c_int, c_int, c_f, c_f, c_int,
                                      c_int, c_u64, c_int, c_p, c_p, c_p]),
    "hicgat_adam_step": (c_int, [c_p, c_p, c_p, c_p, c_i64, c_d, c_d, c_d, c_d, c_i64, c_p]),
    "hicgat_adam_step_table": (c_int, [c_p, c_p, c_p, c_p, c_i64, c_d, c_d, c_d, c_p, c_i64, c_p, c_p]),
    "hicgat_adam_step_table_ex": (c_int, [c_p, c_p, c_p, c_p, c_i64, c_d, c_d, c_d, c_p, c_i64, c_p, c_int, c_p]),
    "hicgat_step_begin": (c_int, [c_p, c_i64, c_p, c_p]),
    "hicgat_step_begin_pack": (c_int, [c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "hicgat_sim_collective": (c_int, [c_f, c_int, c_int, c_p]),
    "hicgat_stream_create": (c_int, [c_int, ctypes.POINTER(c_p)]),
    "hicgat_wall_stamp": (c_int, [c_p, c_int, c_p]),
}


class HicgatUnavailable(RuntimeError):
    """libhicgat.so or the GPU it needs is not available (there is deliberately no fallback)."""


class HicgatError(RuntimeError):
    pass


_lib = None


def load(path=LIB_PATH):
    """Load libhicgat.so and bind every symbol of include/hicgat.h (no GPU needed for this)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HicgatUnavailable(f"{path} not built: run `make -C hic-gnn_amd` (hipcc, gfx950)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib():
    l = load()
    if not torch.cuda.is_available():
        raise HicgatUnavailable("hicgat kernels need an MI355X (torch.cuda.is_available() is False)")
    return l


def check(rc, what):
    if rc != 0:
        msg = load().hicgat_strerror(rc).decode()
        raise HicgatError(f"{what} failed: {msg} ({rc})")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    """The current stream's handle for a launch; inside a graph capture it must be the capture's
    origin or a stream forked into it (``streams.check_launch``)."""
    h = torch.cuda.current_stream(device).cuda_stream
    if _streams.LEDGER.active:
        _streams.check_launch(h)
    return ctypes.c_void_p(h)


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)
