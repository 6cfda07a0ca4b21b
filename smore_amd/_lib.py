"""ctypes binding of libsmore_hip.so (include/smore_hip.h).

The HIP library is the product: there is no Python or CPU fallback.  If the
shared object is missing or fails to load, importing smore_amd raises.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SMORE_LIB") or os.path.join(HERE, "lib", "libsmore_hip.so")   # SMORE_LIB: tuning variants

OK, EINVAL, EHIP, ENOMEM, ESTATE, EIO = range(6)
VM = {"out_degrees": 0, "no_degrees": 1, "degrees": 2}
NM = {"degrees": 0, "in_degrees": 1, "no_degrees": 2}
AT_VERTEX, AT_NEGATIVE, AT_CONTEXT = 0, 1, 2
W, CTX = 0, 1
MODEL = {"line2": 0, "line1": 1, "mf": 2, "bpr": 3, "census": 16}   # census: smore_row_rates of the last census
# exchange rules of the replica exchange (smore_hip.h SMORE_SYNC_*)
SYNC = {"sum": 0, "mean": 1, "adaptive": 2}


def sync_rule(sync):
    """SMORE_SYNC_* of a rule name; booleans are the old mean flag."""
    if isinstance(sync, bool):
        return int(sync)
    return SYNC[sync]


MODE = {"hogwild": 0, "atomic": 1, "serial": 2, "hybrid": 3}
# multi-GPU schedules of the group (smore_hip.h SMORE_SCHED_*)
SCHED = {"replicas": 0, "blocks": 1}
SEM = {"cpp": 0, "go": 1}


class SmoreError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libsmore_hip.so not built (%s); run `make` or __graft_entry__.build()" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    P, i32, i64, u64, dbl = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_double
    sig = {
        "smore_create": (i32, [i32, C.POINTER(P)]),
        "smore_destroy": (None, [P]),
        "smore_last_error": (C.c_char_p, [P]),
        "smore_set_stream": (i32, [P, P]),
        "smore_synchronize": (i32, [P]),
        "smore_version": (C.c_char_p, []),
        "smore_load_edgelist": (i32, [P, C.c_char_p, i32, i32, i32]),
        "smore_set_load_cache": (i32, [P, C.c_char_p]),
        "smore_save_graph": (i32, [P, C.c_char_p]),
        "smore_load_graph": (i32, [P, C.c_char_p, i32, i32]),
        "smore_last_load_info": (i32, [P, C.POINTER(dbl), C.POINTER(i32), C.POINTER(i32)]),
        "smore_set_graph_edges": (i32, [P, i64, i64, P, P, P, i32, i32]),
        "smore_graph_info": (i32, [P, C.POINTER(i64), C.POINTER(i64)]),
        "smore_vertex_name": (C.c_char_p, [P, i64]),
        "smore_get_csr": (i32, [P, P, P]),
        "smore_set_alias": (i32, [P, i32, P, P, i64]),
        "smore_get_alias": (i32, [P, i32, P, P, i64]),
        "smore_get_alias_encoded": (i32, [P, i32, P, P, i64]),
        "smore_alloc_tables": (i32, [P, i32, i32]),
        "smore_init_table_glibc": (i32, [P, i32, u64]),
        "smore_init_table_uniform": (i32, [P, i32, u64]),
        "smore_zero_table": (i32, [P, i32]),
        "smore_set_table": (i32, [P, i32, P, i64, i32]),
        "smore_get_table": (i32, [P, i32, P, i64, i32]),
        "smore_table_device": (i32, [P, i32, C.POINTER(P), C.POINTER(i64)]),
        "smore_train_edges_async": (i32, [P, i32, u64, u64, u64, i32, dbl, dbl, u64, i32]),
        "smore_train_edges": (i32, [P, i32, u64, u64, u64, i32, dbl, dbl, u64, i32]),
        "smore_skipped": (i32, [P, C.POINTER(u64)]),
        "smore_set_hot_threshold": (i32, [P, dbl]),
        "smore_set_semantics": (i32, [P, i32]),
        "smore_set_write_combine": (i32, [P, i32, i32]),
        "smore_write_combine_info": (i32, [P, C.POINTER(i32), C.POINTER(i32)]),
        "smore_gen_powerlaw": (i32, [i64, i64, i32, dbl, u64, P, P]),
        "smore_hot_rows": (i32, [P, C.POINTER(i64), C.POINTER(i64)]),
        "smore_hot_row_ids": (i32, [P, i32, i32, i32, i64, P]),
        "smore_group_set_hot_exchange": (i32, [P, i64, i32]),
        "smore_last_kernel_ms": (C.c_float, [P]),
        "smore_last_mode": (i32, [P]),
        "smore_copy_bandwidth": (i32, [P, u64, i32, C.POINTER(C.c_double)]),
        "smore_last_phase_ms": (i32, [P, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(i32)]),
        "smore_delta_begin": (i32, [P, P, P, P, P, i64]),
        "smore_delta_end": (i32, [P, P, P, P, P, C.c_float, i64]),
        "smore_delta_cycle": (i32, [P, P, P, P, P, C.c_float, i64]),
        "smore_delta_end_rows": (i32, [P, P, P, P, P, P, i64, i64]),
        "smore_delta_cycle_rows": (i32, [P, P, P, P, P, P, i64, i64]),
        "smore_row_rates": (i32, [P, i32, i32, i32, i64, P]),
        "smore_source_parts": (i32, [P, i32, P]),
        "smore_set_source_partition": (i32, [P, i32, i32]),
        "smore_exchange_set_adaptive": (i32, [P, i32, i32, dbl, dbl]),
        "smore_group_set_adaptive": (i32, [P, dbl]),
        "smore_group_set_partition": (i32, [P, i32]),
        "smore_group_set_walk_partition": (i32, [P, i32]),
        "smore_train_deepwalk": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, u64, P, i32]),
        "smore_train_deepwalk_async": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, u64, P, i32]),
        "smore_set_temporal_edges": (i32, [P, i64, P, P, P]),
        "smore_train_ctdne": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, dbl, u64, P, i32]),
        "smore_train_ctdne_async": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, dbl, u64, P, i32]),
        "smore_set_node_types": (i32, [P, P, i32]),
        "smore_train_metapath2vec": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, P, P, i32, u64, P, i32]),
        "smore_train_metapath2vec_async": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, P, P, i32, u64, P, i32]),
        "smore_train_node2vec": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, dbl, dbl, u64, P, i32]),
        "smore_train_node2vec_async": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, dbl, dbl, u64, P, i32]),
        "smore_comm_unique_id": (i32, [P]),
        "smore_comm_init": (i32, [P, i32, i32, P]),
        "smore_exchange_reset": (i32, [P]),
        "smore_exchange_begin": (i32, [P, i32]),
        "smore_exchange_end": (i32, [P]),
        "smore_group_create": (i32, [P, i32, C.POINTER(P)]),
        "smore_group_destroy": (None, [P]),
        "smore_group_size": (i32, [P]),
        "smore_group_ctx": (C.c_void_p, [P, i32]),
        "smore_group_last_error": (C.c_char_p, [P]),
        "smore_group_load_edgelist": (i32, [P, C.c_char_p, i32, i32, i32]),
        "smore_group_set_graph_edges": (i32, [P, i64, i64, P, P, P, i32, i32]),
        "smore_group_set_semantics": (i32, [P, i32]),
        "smore_group_alloc_tables": (i32, [P, i32, i32]),
        "smore_group_broadcast_tables": (i32, [P]),
        "smore_group_train_edges": (i32, [P, i32, u64, u64, u64, i32, dbl, dbl, u64, i32, u64, i32]),
        "smore_group_train_deepwalk": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, u64, P, i32, u64, i32]),
        "smore_group_set_alias": (i32, [P, i32, P, P, i64]),
        "smore_group_set_node_types": (i32, [P, P, i32]),
        "smore_group_set_temporal_edges": (i32, [P, i64, P, P, P]),
        "smore_group_train_metapath2vec": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, P, P, i32, u64, P, i32, u64,
                                                 i32]),
        "smore_group_train_ctdne": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, dbl, u64, P, i32, u64, i32]),
        "smore_group_train_node2vec": (i32, [P, u64, u64, i32, i32, i32, i32, dbl, dbl, dbl, u64, P, i32, u64, i32]),
        "smore_deepwalk_order": (i32, [i64, i32, u64, P]),
        "smore_train_walklets": (i32, [P, u64, u64, i32, i32, i32, i32, i32, dbl, u64, i32]),
        "smore_train_app": (i32, [P, u64, u64, i32, i32, dbl, i32, dbl, u64, P, i32]),
        "smore_train_hpe": (i32, [P, u64, u64, u64, i32, i32, dbl, dbl, u64, i32]),
        "smore_train_walklets_async": (i32, [P, u64, u64, i32, i32, i32, i32, i32, dbl, u64, i32]),
        "smore_train_app_async": (i32, [P, u64, u64, i32, i32, dbl, i32, dbl, u64, P, i32]),
        "smore_train_hpe_async": (i32, [P, u64, u64, u64, i32, i32, dbl, dbl, u64, i32]),
        "smore_group_train_walklets": (i32, [P, u64, u64, i32, i32, i32, i32, i32, dbl, u64, i32, u64, i32]),
        "smore_group_train_app": (i32, [P, u64, u64, i32, i32, dbl, i32, dbl, u64, P, i32, u64, i32]),
        "smore_group_train_hpe": (i32, [P, u64, u64, u64, i32, i32, dbl, dbl, u64, i32, u64, i32]),
        "smore_sample_edges": (i32, [P, i32, u64, u64, i32, u64, P]),
        "smore_train_pairs": (i32, [P, P, P, i64, i32, dbl, u64, u64, i32]),
        "smore_pairs_rows": (i32, [P, P, P, i64, i32, u64, u64, P, C.POINTER(i64), P, C.POINTER(i64)]),
        "smore_set_rows": (i32, [P, i32, P, i64, P]),
        "smore_get_rows": (i32, [P, i32, P, i64, P]),
        "smore_train_pairs_rows": (i32, [P, P, P, i64, i32, dbl, u64, u64, i32, P, i64, P, P, i64, P]),
        "smore_train_pairs_rows_mt": (i32, [P, P, P, i64, i32, dbl, u64, u64, i32, P, i64, P, P, i64, P]),
        "smore_pairs_combine_stats": (i32, [P, P, P]),
        "smore_census_begin": (i32, [P]),
        "smore_census_end": (i32, [P, dbl]),
        "smore_set_walk_owner": (i32, [P, i64, i64]),
        "smore_walk_parts": (i32, [P, i32, P]),
        "smore_group_set_schedule": (i32, [P, i32]),
        "smore_set_comm_timeout": (i32, [dbl]),
        "smore_block_setup": (i32, [P, i32, i32, i32, i32, i32]),
        "smore_block_info": (i32, [P, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
        "smore_block_bounds": (i32, [P, P, P]),
        "smore_block_mass": (i32, [P, P]),
        "smore_block_part_mass": (i32, [P, P]),
        "smore_block_neg_scale": (i32, [P, i32, P]),
        "smore_block_set_hubs": (i32, [P, i64]),
        "smore_block_hubs": (i32, [P, P, P, P, P]),
        "smore_block_hubs_load": (i32, [P]),
        "smore_block_hubs_store": (i32, [P]),
        "smore_block_hub_scales": (i32, [P, dbl, dbl, P]),
        "smore_block_cell_launches": (i32, [P]),
        "smore_block_walks_generate": (i32, [P, i32, u64, u64, u64, u64, i32, i32, i32, i32, i32, dbl, u64, P, u64,
                                             i32]),
        "smore_block_walks_emit": (i32, [P]),
        "smore_block_walks_buffer": (i32, [P, P, P, P]),
        "smore_block_train_walks_part_async": (i32, [P, i32, i32, i32]),
        "smore_block_counts": (i32, [P, u64, P]),
        "smore_block_train_edges_async": (i32, [P, i32, u64, u64, u64, i32, dbl, u64, i32]),
        "smore_block_sample_edges": (i32, [P, i32, u64, u64, u64, i32, P]),
        "smore_block_prepare_walks": (i32, [P, i32, u64, u64, i32, i32, i32, i32, i32, dbl, u64, P, u64, i32]),
        "smore_block_train_walks_async": (i32, [P, i32]),
        "smore_block_walk_records": (i32, [P, i32, C.POINTER(u64)]),
        "smore_block_walk_records_copy": (i32, [P, i32, P, u64, C.POINTER(u64), C.POINTER(i32)]),
        "smore_save_weights": (i32, [P, i32, C.c_char_p, i32]),
        "smore_load_pretrain": (i32, [P, i32, C.c_char_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    L._signatures = sig
    return L


lib = _load()


def check(ctx, rc, what=""):
    if rc != OK:
        msg = lib.smore_last_error(ctx).decode() if ctx else ""
        raise SmoreError("%s failed (status %d): %s" % (what, rc, msg))


def ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)
