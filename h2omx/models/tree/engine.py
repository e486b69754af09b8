"""Level-wise histogram tree builder (the GBM / XGBoost / DRF hot loop).

``HipTreeBuilder`` drives the gfx950 kernels of ``csrc/tree_kernels.hip``.
Per tree level it enqueues, on the current HIP stream and without any host
synchronisation::

    hist_build (LDS)  ->  hist_reduce (fp64)  ->  [all_reduce over RCCL]
    -> split_find (node x feature)  ->  level_finalize  ->  partition

The decision of which nodes split, how children are numbered and which child
is histogrammed (the smaller one; its sibling comes from parent - child) is
taken on the device, so the host never waits for the GPU inside a tree.

``RefTreeBuilder`` (``h2omx/reference/tree.py``) implements the same algorithm with
NumPy on the CPU; it is the test oracle and the CPU plumbing path.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from ... import ops
from .binning import BinnedMatrix
from ...utils.trace import PhaseTimer
from .structs import (FEAT_BEST_BYTES, NODE_LINK_BYTES, PART_INFO_BYTES, TREE_NODE_DTYPE, GradParams,
                      SplitParams, check_layout, interaction_masks)


@dataclass
class TreeParams:
    max_depth: int = 5
    min_rows: float = 10.0
    min_child_weight: float = 0.0
    reg_lambda: float = 0.0
    reg_alpha: float = 0.0
    gamma: float = 0.0
    min_split_improvement: float = 1e-5
    learn_rate: float = 0.1
    learn_rate_annealing: float = 1.0   # H2O GBM: iteration t uses learn_rate * annealing^t
    mode: int = 0            # 0: H2O squared error on residuals, 1: XGBoost second order
    leaf_mode: int = 0       # 0: Newton (-G/(H+lambda)), 1: mean (DRF)
    col_sample_rate: float = 1.0
    col_sample_rate_per_tree: float = 1.0
    mtries: int = 0
    max_abs_leaf: float = 0.0
    seed: int = 0
    # per-feature monotone constraint (-1 / 0 / +1), None = unconstrained
    monotone: tuple | None = None
    # interaction constraints: tuple of feature-index tuples (features of one set
    # may share a root path; unlisted features only with themselves), None = off
    interactions: tuple | None = None
    # per-node histogram rule (binning.PER_NODE_MODES: 0 every fine bin, 1
    # UniformAdaptive, 2 Random, 3 RoundRobin) with H2O's nbins_top_level / nbins;
    # modes 1-3 need BinnedMatrix.frange (binning.adaptive_ranges)
    hist_mode: int = 0
    hist_top: int = 1024
    hist_nbins: int = 20
    extra: dict = field(default_factory=dict)


def tree_capacity(max_depth: int) -> int:
    return (1 << (max_depth + 1)) - 1


class HipTreeBuilder:
    """Builds one tree per call entirely with enqueued HIP kernels.

    Per tree: quantisation scales from the gradient maxima (written by the
    boost kernel into ``stat_max``) -> per level {hist_build, hist_reduce,
    [RCCL all-reduce], split_find, level_finalize, partition} -> exact leaf
    sums (leaf_stats, [all-reduce], leaf_finalize).
    """

    # LDS histogram bytes per workgroup / threads per workgroup / target grid
    # (the sweeps that fixed them: profiles/r3/hist_threads_ab.txt,
    # profiles/r4/hist_knobs_11m_r4o.txt)
    LDS_BUDGET = 64 * 1024
    # 1024-thread workgroups, 256 of them (one per CU) on shallow levels: HIGGS 11M
    # depth 5 0.886 vs 0.917 ms/tree for 512 x 512 threads (half the partial slabs
    # to reduce; 384 / 512 workgroups of 1024 threads: 1.13 / 1.08), XGBoost / DRF
    # unchanged (profiles/r3/hist_threads_ab.txt)
    THREADS = 1024
    TARGET_WGS = 512
    ROWS_PER_LANE = 16
    # rows per workgroup chunk: bounds the fixed-point headroom, so the gradient
    # resolution is 2^30 / (largest chunk) levels (see tree_begin)
    ROWS_CAP = 262144
    SYNC_NODE_CAP = 4096   # above this many potential nodes the host reads the real count
    # (Removed A/B variants that measured slower and no longer exist: the
    # wave-compacted column gather (profiles/compact_hist_p9.txt), the
    # row-major built-row gather (profiles/r3/hist_rm_ab.txt), the route_kernel
    # routing pass, split_find_fin / split_level fused splits
    # (profiles/r3/hist_threads_ab.txt) and the segment-ordered code-row moves
    # (profiles/r4/drf/move_rows_ab.txt).)
    SEG_TARGET_CHUNKS = 1024   # level-0 histogram chunks (2 resident 57 KB workgroups per CU)
    # segmented-histogram LDS per workgroup (feature group size): small histograms (<= 64 bins)
    # run more, narrower groups - DRF 10M x 100 depth 20: 64 / 32 / 24 / 16 / 12 / 8 / 4 KB ->
    # 13.68 / 13.21 / 13.16 / 12.71 / 12.73 / 12.81 / 12.85 ms/tree (profiles/r6/drf_switches_r6o.txt
    # r6bh-r6bj); 255-bin histograms keep 64 KB (16 KB: 19.4 vs 19.0 ms/tree, r6bk)
    SEG_LDS_BUDGET = 16 * 1024
    SEG_LDS_BUDGET_WIDE = 64 * 1024
    # seg engine: scan hist up to this many slots - the root only: from level 1 on the
    # segmented build reads the built children's in-bag rows instead of streaming all
    # rows (DRF 10M x 100 depth 20: levels 2-5, histograms + partitions 2002 -> 1628 us,
    # 17.51 -> 16.73 ms/tree; profiles/r6/drf_deep_ab_r6.txt r6ag / r6ah)
    SCAN_SLOTS = 1
    MEAN_LEAVES_NO_H = True   # mean-leaf trees pass no h to the partitions (their H sums are unused)
    # bagged deep trees: the root segment holds only in-bag rows (bag_compact_kernel); set per
    # booster (bag_compact: sample_rate < 1)
    BAG_COMPACT = True
    bag_compact = False
    DEEP_DEPTH = 10
    FUSE_MAX_DEPTH = 8
    FUSE_MAX_PREV = 4
    CLOSE_SINGLE_BLOCK = 2048
    # segmented engine, single rank: levels with >= this many potential nodes build each
    # node's eligible-feature histograms directly and scan them in LDS (seg_direct_kernel:
    # no parent histograms / subtraction); 0 = off.  Multi-rank runs keep the all-reduced
    # subtraction path (direct histograms are rank-local).  DRF 10M x 100 depth 20: 512 / 1024 /
    # 2048 / 4096 -> 15.66 / 14.85 / 14.66 / 14.74 ms/tree (profiles/r6/drf_switches_r6o.txt r6ap / r6aq)
    DIRECT_MIN_NODES = 2048
    # ... and only when a node has at most this many eligible features on average
    DIRECT_MAX_ELIG = 32.0
    # direct levels whose average node holds fewer rows than this run one wave per node
    # (seg_direct_wave_kernel, F <= 256) instead of one workgroup per node (DRF 10M x 100
    # depth 20: 128 / 256 / 512 / 1024 / 2048 -> 16.13 / 15.13 / 14.85 / 15.05 / 15.76 ms/tree,
    # profiles/r6/drf_switches_r6o.txt r6an / r6ao)
    DIRECT_WAVE_ROWS = 512
    # segmented partition: levels of at least this many potential nodes run one wave per row chunk
    # (part_count_wave / part_scatter_wave: 64-ary chunk -> node search, stored row directions)
    PART_WAVE_NODES = 2048
    # direct levels of large nodes: one workgroup per row chunk (False: one per node)
    DIRECT_CHUNKED = True
    # partition grid: 1024 x 256 lanes (sweep on HIGGS 11M: 512 1.56, 1024 1.47,
    # 2048 1.49, 4096 1.55 ms/tree)
    PART_BLOCKS = 1024
    # path switches (class attributes: the GPU tests flip them with monkeypatch to
    # pin the alternatives bit-identical): fused routing, 16-bit packed rows,
    # level 0 with the gradient pass fused in (off: see can_fuse_grad), chained
    # tree_begin in graph replay
    FUSE_ROUTE = True
    PK32 = True
    FUSE_GRAD = False
    CHAIN_BEGIN = True
    # partition workgroups spread their leaf-sum folds over this many slices
    # (same-address atomic contention; profiles/r6/partition_atomics_r6g.txt)
    LEAF_REPS = 16
    # level finalisation in the last workgroup of the level's reduce + split scan:
    # N-rank (P2P) levels -3 % on the loopback-8 proxy; one rank neutral
    # (headline / 1.375M shard within noise, profiles/r6/fused_fin_ab_r6e.txt),
    # so the single-rank level keeps the separate finalisation launch
    FUSE_FIN = True
    FUSE_FIN_LOCAL = False
    # segmented engine: part_scatter moves each row's (g, s2) into segment order with it
    PERMUTE_GS = True
    # direct levels of <= 16 eligible features store them per row for the partition
    ECODES = True
    # levels of more than 8192 nodes finalise in count / scan / write tiles (False: one workgroup)
    LF_MULTI_BLOCK = True
    # row-chunk direct levels (one rank, dmode 2): the first one and every k-th
    # after it transpose the live rows' codes into column-major planes in
    # segment order (seg_colmajor_kernel); the ones in between move only
    # positions.  Wave-per-node levels read the row-major codes (their scan is
    # issue-bound, profiles/r6/drf_pmc_r6i.txt).  0 = off: once out-of-bag rows left the
    # segments (BAG_COMPACT) and direct levels start at 2048 nodes, the one transpose no
    # longer pays (DRF 10M x 100 depth 20: 13.95 -> 13.75 ms/tree, profiles/r6/drf_switches_r6o.txt
    # r6bc / r6bd; it did on the earlier pipeline: level 10 1121 -> 525 us, r6j)
    COLMAJOR_EVERY = 0

    def __init__(self, bm: BinnedMatrix, params: TreeParams, comm=None):
        if not bm.codes.is_cuda:
            raise ValueError("HipTreeBuilder needs device-resident codes")
        self.lib = ops.tree_lib()
        check_layout(self.lib)
        self.bm = bm
        self.p = params
        self.comm = comm
        self.dev = bm.codes.device
        self.F = bm.F
        self.nbt = bm.nbt
        self.per_node = self.F * 2 * self.nbt  # int64 per node histogram (G_q, S_q planes)
        if params.max_depth < 1:
            raise ValueError("max_depth must be >= 1")
        self.capacity = tree_capacity(min(params.max_depth, 24))
        d = self.dev
        self.ctl = torch.zeros((2, 4), dtype=torch.int32, device=d)
        self.ctl_init = torch.tensor([1, 1, 0, 1], dtype=torch.int32, device=d)
        self.link_init = torch.tensor([0, -1, -1, 0], dtype=torch.int32, device=d)
        self._bufs: dict[str, torch.Tensor] = {}
        self.tree_buf = torch.zeros((self.capacity * TREE_NODE_DTYPE.itemsize,), dtype=torch.uint8, device=d)
        self.nid = torch.full((bm.npad,), -1, dtype=torch.int32, device=d)
        self.stat_max = torch.zeros((4,), dtype=torch.int32, device=d)   # float bits of max|g|, max h, max w
        self.stat_slab = torch.zeros((int(self.lib.h2omx_stat_blocks()) * 4,), dtype=torch.int32, device=d)
        self.qscale = torch.zeros((16,), dtype=torch.float64, device=d)
        self.qscale[8] = float(bm.n)          # live rows of this rank (implicit-root levels)
        self.leaf_acc = torch.zeros((self.capacity * 3,), dtype=torch.int64, device=d)
        # per-row packed quantised (g, s) of the current tree and next-level build
        # slot (scan engine): written at level 0 / by partition, read by deeper levels
        self.pk = torch.empty((bm.npad,), dtype=torch.int64, device=d)
        self.slot16 = torch.empty((bm.npad,), dtype=torch.int16, device=d)
        self.part_blocks = min(int(self.lib.h2omx_partition_blocks()), self.PART_BLOCKS)
        self._sp = SplitParams()
        # monotone constraints: per-feature sign + every node's value interval
        # (written by the parent's level finalisation, read by its children)
        self.mono = self.gbound = None
        if params.monotone is not None and any(int(m) != 0 for m in params.monotone):
            if len(params.monotone) != self.F:
                raise ValueError(f"monotone has {len(params.monotone)} entries for {self.F} features")
            self.mono = torch.tensor([int(np.sign(m)) for m in params.monotone], dtype=torch.int8, device=d)
            self.gbound = torch.zeros((2 * self.capacity,), dtype=torch.float64, device=d)
        # interaction constraints: per-feature set masks + every node's state
        # (compatible sets, solo feature), written by the parent's finalisation
        self.ifsets = self.istate = None
        if params.interactions:
            fs = interaction_masks(params.interactions, self.F)
            self.ifsets = torch.from_numpy(fs.view(np.int64).copy()).to(d)
            self.istate = torch.zeros((2 * self.capacity,), dtype=torch.int64, device=d)
            self.istate[0], self.istate[1] = -1, -2     # root: every set, empty path
        # categorical group splits: feature flags on the device, the tree's left-set
        # bitsets ([capacity][8] uint32, one tree at a time, snapshotted with tree_buf)
        # and the per-(node, feature) scan bitsets (fbcat, per level)
        self.catf = bm.catf
        self.treecat = (torch.zeros((self.capacity * 8,), dtype=torch.int32, device=d)
                        if self.catf is not None else None)
        # per-node histogram rules read the fine edges and every feature's
        # (min, max, exact, integer) in the split scan
        self._frange = None
        if params.hist_mode:
            if getattr(bm, "frange", None) is None:
                raise ValueError("TreeParams.hist_mode needs BinnedMatrix.frange (binning.adaptive_ranges)")
            self._frange = bm.frange.to(d).float().contiguous()
        self.stats = {"host_syncs": 0}
        self.timer = PhaseTimer(device=d)
        # global index of this rank's first row: the stochastic-rounding dither and
        # bagging hash use global row ids, so a multi-GPU model is bit-identical to
        # the single-GPU model on the concatenated rows
        self.row_base, n_global = global_rows(bm.n, comm)
        self.plans = {}
        # largest workgroup row chunk over every plan this tree can use: sets the
        # fixed-point resolution (finer for smaller chunks), identical across levels.
        # Evaluated on the GLOBAL row count (every rank, and a 1-rank run on the
        # same rows, derives the same scale: strong-scaled runs are bit-identical to
        # one GPU); the local plans are then held to chunks <= this (see _plan).
        self.max_rows_per_wg = None
        g_units = max(1, -(-n_global // 64) * 64) // self.ROWS_PER_LANE
        cands = [self._choose(1 << k, g_units) for k in range(0, 13)] + [self._choose(1 << 20, g_units)]
        self.max_rows_per_wg = max(self.ROWS_PER_LANE * math.ceil(g_units / c["wgpg"]) for c in cands)
        # >= 2^16 rows per workgroup bounds the per-row fixed-point values to 16 bits
        # (tree_begin: |G_q| <= 2^14, S_q <= 2^15): the packed rows are then stored in
        # 32 bits (hist_build PKM 3/4), halving what every deep-level feature group re-reads
        # (self.pk32, set once the ranks agree on max_rows_per_wg below)
        # fused routing (scan engine, shallow trees): level d's partition runs inside
        # level d+1's histogram kernel (node ids double-buffered), and the last level's
        # partition adds the exact sums of every row, early leaves included, into a
        # whole-tree LDS window (needs the tree capacity to fit it: depth <= 8)
        self.fuse_route = params.max_depth <= self.FUSE_MAX_DEPTH and self.FUSE_ROUTE
        # scan engine with fused routing: levels 0 / 1 take "every live row is in the
        # root" from the row count instead of a node-id stream, so boost_update no
        # longer resets nid and levels 0 / 1 skip reading it (needs >= 2 levels: a
        # depth-1 tree's final partition reads level 0's ids)
        self.implicit_root = (self.fuse_route and not getattr(self, "segmented", False)
                              and params.max_depth >= 2)
        self.nid2 = torch.full((bm.npad,), -1, dtype=torch.int32, device=d) if self.fuse_route else None
        self.ticket = torch.zeros((4,), dtype=torch.int32, device=d)
        # graph replay (boost.TreeGraph): tree_begin takes the tree index (dither salt,
        # qscale[9]) from this device counter instead of the host argument, and advances it
        self.tree_ctr = None
        # Engine choice (both build bit-identical trees):
        # * scan: every level streams all rows; best for shallow trees (HIGGS depth 5:
        #   1.52 vs 1.90 ms/tree for the segmented engine, profiles/seg_vs_scan_s1.txt)
        #   but each level costs at least one full pass per slot pass, so deep trees
        #   with thousands of nodes per level need hundreds of passes.
        # * seg (row-partitioned): a level only touches the rows of the nodes it
        #   builds; the root still uses the scan histogram kernel (<= SCAN_SLOTS
        #   built nodes), deep levels the per-node-chunk kernel.  Default for trees
        #   deeper than DEEP_DEPTH (DRF's default max_depth 20).
        eng = os.environ.get("H2OMX_TREE_ENGINE", "auto")
        self.segmented = eng == "seg" or (eng == "auto" and params.max_depth > self.DEEP_DEPTH)
        # leaf-sum replicas of the scan engine's partitions ([reps][3 x capacity],
        # qscale[10]; csrc/tree_kernels.hip leaf_reps): small trees only
        self.leaf_reps = self.LEAF_REPS if (not self.segmented and self.capacity <= 4096) else 1
        if self.leaf_reps > 1:
            self.leaf_acc = torch.zeros((self.leaf_reps * self.capacity * 3,), dtype=torch.int64, device=d)
        self.qscale[10] = float(self.leaf_reps)
        if self.segmented:
            self.fuse_route, self.nid2 = False, None
            self.implicit_root = False
            self.pc_rows = int(self.lib.h2omx_pc_rows())
            hc = -(-bm.n // self.SEG_TARGET_CHUNKS)
            self.hc_rows = min(self.ROWS_CAP, max(2048, -(-hc // 256) * 256))
            # the scale covers the chunk size a 1-rank run on all rows would use
            hc_g = -(-n_global // self.SEG_TARGET_CHUNKS)
            self.max_rows_per_wg = max(self.max_rows_per_wg, self.hc_rows,
                                       min(self.ROWS_CAP, max(2048, -(-hc_g // 256) * 256)))
            budget = self.SEG_LDS_BUDGET if self.nbt <= 64 else self.SEG_LDS_BUDGET_WIDE
            fg = max(1, min(self.F, budget // (self.nbt * 8)))
            groups = math.ceil(self.F / fg)
            if groups > 1:
                fg = max(4, (math.ceil(self.F / groups) + 3) // 4 * 4)
                groups = math.ceil(self.F / fg)
            self.seg_fg, self.seg_groups = fg, groups
            self.seg_threads = 512
            self.codes_rm = bm.codes_rm
            self.idx = [torch.empty((max(bm.n, 1),), dtype=torch.int32, device=d) for _ in range(2)]
        # int16 node ids between the fused-routing levels (2 bytes a row each way
        # instead of 4)
        self.nid16 = None
        if self.fuse_route and self.implicit_root and self.ROWS_PER_LANE == 16 and self.capacity < 32767:
            self.nid16 = (torch.full((bm.npad,), -1, dtype=torch.int16, device=d),
                          torch.full((bm.npad,), -1, dtype=torch.int16, device=d))
        # the fixed-point scales (tree_begin) derive from max_rows_per_wg: every rank
        # quantises with the SAME scale (derived from the global row count above), so
        # the summed int64 histograms are in one unit
        self.pk32 = self.max_rows_per_wg >= 65536 and self.PK32

    # -- buffers -----------------------------------------------------------
    def _ticket_buf(self, numel: int) -> torch.Tensor:
        """zeroed per-node arrival counters; kernels reset the entries they use"""
        t = getattr(self, "_tickets", None)
        if t is None or t.numel() < numel:
            t = self._tickets = torch.zeros(max(numel, 1024), dtype=torch.int32, device=self.dev)
        return t

    def _lf_tiles(self, max_nodes: int) -> int:
        """tile scratch of the multi-block level finalisation (0 = single workgroup)"""
        if not self.LF_MULTI_BLOCK:
            return 0
        return self._buf("lf_tiles", max_nodes // 1024 + 2, torch.int32).data_ptr()

    def _buf(self, name: str, numel: int, dtype) -> torch.Tensor:
        b = self._bufs.get(name)
        if b is None or b.numel() < numel:
            b = torch.empty((max(numel, 1),), dtype=dtype, device=self.dev)
            self._bufs[name] = b
        return b

    # -- planning ------------------------------------------------------------
    DEEP_LDS_BUDGET = 128 * 1024
    DEEP_MIN_GROUPS = 4
    # level 0 of the scan engine: histograms in 8 interleaved lane copies
    # (hist_build COP: fewer LDS bank conflicts, 8x the LDS per feature, so
    # feature groups of DEEP_LDS_BUDGET); 1 = plain slices
    L0_COPIES = 8

    def plan_l0(self):
        key = ("l0", self.L0_COPIES)
        if key not in self.plans:
            self.plans[key] = self._plan(1, self.DEEP_LDS_BUDGET, self.THREADS, mult=self.L0_COPIES)
        return self.plans[key]

    # grids that overflow one round of resident workgroups are widened to fill
    # their last round: the chunk cap (ROWS_CAP) puts Airlines-shape 18.75M rows
    # at 72 x 4 = 288 one-per-CU workgroups, so 32 of them ran alone in a
    # second round
    N_CUS = 256
    MIN_GROUPS = 1
    # single rank: slab reduction + split scan in one launch per pass (reduce_split)
    # persistent workgroups of the N-rank fused level (<= 256 P2P flag slots)
    P2P_BLOCKS = 256
    MAX_WG_THREADS_PER_CU = 2048      # 32 waves per CU

    def _fill_rounds(self, wgpg: int, n_groups: int, lds_bytes: int, threads: int, units: int) -> int:
        per_cu = max(1, min((160 * 1024) // max(1, lds_bytes + 3072), self.MAX_WG_THREADS_PER_CU // threads))
        resident = self.N_CUS * per_cu
        total = n_groups * wgpg
        if total <= resident:
            return wgpg
        rounds = math.ceil(total / resident)
        fill = (rounds * resident // n_groups) // 8 * 8
        # keep >= 1 row unit per lane
        if fill > wgpg and fill * threads <= units:
            return fill
        return wgpg

    # small-shard grid widening and round filling (class flags: the planner tests
    # compare against the plans without them)
    SMALL_SHARD = True
    FILL_ROUNDS = True

    def _plan(self, max_slots: int, budget: int, threads: int, units: int | None = None, mult: int = 1):
        per_slot_feat = self.nbt * 8 * mult
        F = self.F
        if max_slots * per_slot_feat <= budget:
            slot_cnt = max_slots
            fg_max = max(1, min(F, 256, budget // (max_slots * per_slot_feat)))
            n_groups = math.ceil(F / fg_max)
            fg = math.ceil(F / n_groups)
            passes = 1
        else:
            fg, n_groups = 1, F
            slot_cnt = max(1, budget // per_slot_feat)
            passes = math.ceil(max_slots / slot_cnt)
        if passes == 1 and self.MIN_GROUPS > n_groups and mult == 1:
            fg = math.ceil(F / min(F, self.MIN_GROUPS))
            n_groups = math.ceil(F / fg)
        if units is None:
            units = self.bm.npad // self.ROWS_PER_LANE

        def target(t: int) -> int:
            return max(8, (self.TARGET_WGS * 512 // t // n_groups) // 8 * 8)

        def grid(t: int, upl: int) -> int:
            return min(target(t), max(8, (units // (t * upl)) // 8 * 8))   # keep >= upl row units per lane

        wgpg = grid(threads, 2)
        if self.SMALL_SHARD and n_groups * wgpg < self.N_CUS and wgpg < target(threads):
            # small shards (strong scaling: 11M / 8 ranks = 86K row units) put the
            # 2-units-per-lane grid on a fraction of the CUs (level 1: 40 of 256
            # workgroups); spread them over every CU with 1 unit per lane and, if
            # still short, more feature groups (the re-read rows of a small shard
            # stay in L2 / MALL; narrower 512 / 256-thread workgroups measured slower)
            wgpg = grid(threads, 1)
            if n_groups * wgpg < self.N_CUS and passes == 1:
                ng = min(F, math.ceil(self.N_CUS / wgpg))
                if ng > n_groups:
                    fg = math.ceil(F / ng)
                    n_groups = math.ceil(F / fg)
                    wgpg = grid(threads, 1)
        cap =self.ROWS_CAP if self.max_rows_per_wg is None else min(self.ROWS_CAP, self.max_rows_per_wg)
        min_wgpg = math.ceil(math.ceil(units / (cap // self.ROWS_PER_LANE)) / 8) * 8
        wgpg = max(wgpg, min_wgpg)
        if self.FILL_ROUNDS:
            wgpg = self._fill_rounds(wgpg, n_groups, slot_cnt * fg * per_slot_feat, threads, units)
        return dict(slot_cnt=slot_cnt, fg=fg, n_groups=n_groups, passes=passes, wgpg=wgpg, threads=threads)

    def plan_level(self, max_slots: int):
        """Feature grouping / slot passes / grid for a level with max_slots built nodes.
        Shallow levels use 64 KB / 512-thread workgroups (2 per CU); levels
        that would need >= 4 feature groups switch to 128 KB / 1024 threads
        (1 per CU) so each row chunk is re-read by fewer groups."""
        key = max_slots
        if key in self.plans:
            return self.plans[key]
        plan = self._choose(max_slots)
        self.plans[key] = plan
        return plan

    def _choose(self, max_slots: int, units: int | None = None):
        """plan_level's choice for ``units`` row units (default: this rank's)."""
        lo, hi = self.LDS_BUDGET, self.DEEP_LDS_BUDGET
        plan = self._plan(max_slots, lo, self.THREADS, units)
        if hi > lo and plan["n_groups"] >= self.DEEP_MIN_GROUPS:
            deep = self._plan(max_slots, hi, 1024, units)
            if deep["n_groups"] < plan["n_groups"] or deep["passes"] < plan["passes"]:
                plan = deep
        return plan

    def _fused_level(self, d: int) -> bool:
        """Level d >= 1 routes its rows inside its histogram kernel when the
        previous level has at most FUSE_MAX_PREV nodes (one coalesced code load
        per previous node and row unit; wider levels keep a routing pass)."""
        return (1 << (d - 1)) <= self.FUSE_MAX_PREV

    def _params(self, tree_index: int):
        p, sp = self.p, self._sp
        sp.mode, sp.leaf_mode, sp.F, sp.is_last_level = p.mode, p.leaf_mode, self.F, 0
        sp.min_rows, sp.min_child_weight = p.min_rows, p.min_child_weight
        sp.lambda_, sp.alpha, sp.gamma = p.reg_lambda, p.reg_alpha, p.gamma
        sp.min_split_improvement, sp.learn_rate, sp.max_abs_leaf = p.min_split_improvement, p.learn_rate, p.max_abs_leaf
        sp.seed, sp.tree_index = p.seed & 0xFFFFFFFF, tree_index
        sp.col_rate, sp.mtries = p.col_sample_rate, p.mtries
        sp.mono = self.mono.data_ptr() if self.mono is not None else None
        sp.gbound = self.gbound.data_ptr() if self.gbound is not None else None
        sp.ifsets = self.ifsets.data_ptr() if self.ifsets is not None else None
        sp.istate = self.istate.data_ptr() if self.istate is not None else None
        sp.catf = self.catf.data_ptr() if self.catf is not None else None
        sp.treecat = self.treecat.data_ptr() if self.treecat is not None else None
        sp.fbcat = None
        sp.hist_mode, sp.hist_top, sp.hist_nbins = p.hist_mode, p.hist_top, p.hist_nbins
        sp.edges = self.bm.edges.data_ptr() if p.hist_mode else None
        sp.frange = self._frange.data_ptr() if p.hist_mode else None
        return ctypes.addressof(sp)

    def _cat_level(self, max_nodes: int) -> None:
        """Point SplitParams::fbcat at a [max_nodes][F][8] scratch for this level."""
        if self.catf is not None:
            self._sp.fbcat = self._buf("fbcat", max_nodes * self.F * 8, torch.int32).data_ptr()

    # -- one tree ------------------------------------------------------------
    def can_fuse_grad(self, dist: str, weighted: bool, sample_rate: float) -> bool:
        """Level 0 can run the gradient pass itself (hist_build PKM 5): scan
        engine with the implicit root, one tree per iteration, no weights /
        bagging, and a distribution whose gradients have fixed bounds
        (GRAD_BOUNDS: every engine quantises those with the bound scales, so
        fused and separate gradient passes build bit-identical trees)."""
        return (not self.segmented and self.implicit_root and not weighted
                and sample_rate >= 1.0 and dist in GRAD_BOUNDS
                and self.FUSE_GRAD)

    def build(self, g: torch.Tensor, h: torch.Tensor, w: torch.Tensor | None, tree_index: int,
              tree_fmask: torch.Tensor | None = None, grad_fuse: dict | None = None,
              stat: torch.Tensor | None = None, chain: bool = False) -> torch.Tensor:
        """Grow one tree from per-row (g, h, w).  Preconditions (established by
        the boost / softmax kernels): ``self.nid`` is 0 for rows of the tree and
        INT_MIN for padding; ``self.stat_max`` holds this tree's maxima.
        Returns the device tree buffer (``TREE_NODE_DTYPE`` heap of capacity
        nodes; unreachable records are garbage).  ``self.stat_max`` must hold
        this tree's gradient maxima (see :meth:`reduce_stats`).

        ``chain`` (graph replay, fixed bounds ``stat``): this tree's begin was
        done by the previous tree's leaf finalisation (or :meth:`begin`), and
        this one's leaf finalisation begins the next tree."""
        # ``stat``: fixed gradient bounds (stat_max image, identical on every rank)
        # used instead of this tree's maxima: no maxima reduction, no all-reduce
        if grad_fuse is not None:
            stat = grad_fuse["bounds"]      # see can_fuse_grad
        smax = self.stat_max if stat is None else stat
        if self.segmented:
            return self._build_seg(g, h, w, tree_index, tree_fmask, smax, stat is not None)
        lib, bm, p = self.lib, self.bm, self.p
        st = ops.stream(self.dev)
        P = ops.P
        F, nbt = self.F, self.nbt
        spp = self._params(tree_index)
        sp = self._sp
        comm = self.comm if (self.comm is not None and self.comm.world_size > 1) else None
        # one-shot P2P transport: N-rank levels exchange their histogram rows inside
        # reduce_split_p2p and the leaf sums inside leaf_finalize_p2p (one launch
        # each, as on one rank); without it (RCCL / gloo) the level all-reduces `built`
        p2p = getattr(comm, "p2p", None) if comm is not None else None

        if comm is not None and stat is None:   # fixed bounds are the same on every rank
            comm.all_reduce_(smax, "max")
        s2 = w if p.mode == 0 else h
        link = [self._buf("link0", 4, torch.int32), None]
        # scales + level-0 control block/link + zeroed leaf sums in one launch
        T = self.timer.phase
        if not chain:
            with T("tree_begin"):
                self.begin(smax, tree_index)
        # level 0 reads the packed rows the previous step's boost_update quantised
        # for this tree (chained graph steps, see can_pack_in_boost)
        pk_boost = chain and self.pk_in_boost
        full_prev = None
        max_depth = p.max_depth
        final_ctl = self.ctl[max_depth % 2]
        max_nodes = 1
        fuse = self.fuse_route
        # int16 node-id streams between the fused levels (NID16): the final
        # partition writes the int32 leaf ids boost_update reads into self.nid
        nid16 = self.nid16 is not None
        nid_buf = self.nid16 if nid16 else (self.nid, self.nid2)
        part_prev = None
        for d in range(max_depth):
            cur, nxt = d % 2, (d + 1) % 2
            ctl_cur, ctl_nxt = self.ctl[cur], self.ctl[nxt]
            if max_nodes > self.SYNC_NODE_CAP:
                n_now, s_now = [int(v) for v in ctl_cur[:2].tolist()]
                self.stats["host_syncs"] += 1
                if n_now == 0:
                    final_ctl = ctl_cur     # tree finished early: ctl_cur holds its final TOTAL
                    break
                max_nodes, max_slots = n_now, s_now
            else:
                max_slots = 1 if d == 0 else max(1, max_nodes // 2)
            last = d == max_depth - 1
            plan = self.plan_level(max_slots)
            l0_copies = d == 0 and grad_fuse is None and self.L0_COPIES in (4, 8)
            if l0_copies:
                plan = self.plan_l0()
            built = self._buf("built", max_slots * self.per_node, torch.int64)
            full_cur = None if last else self._buf(f"full{cur}", max_nodes * self.per_node, torch.int64)
            sp.depth = d
            sp.children_leaves = 1 if last else 0
            self._cat_level(max_nodes)
            # N ranks over P2P: the level's reduce-scatter runs inside the fused
            # reduce + split scan when the level is one histogram pass on EVERY
            # rank (the slot budget alone decides that - rank-independent - while
            # feature groups / grids follow each rank's row count), the rows pushed
            # to one owner fit a parity of the symmetric buffer and the level's
            # split records fit its split table (csrc/tree_kernels.hip)
            fuse_p2p = (p2p is not None
                        and max_slots * nbt * 8 <= self.LDS_BUDGET
                        and max_slots * -(-F // p2p.world) * p2p.world * 2 * nbt * 8 <= p2p.cap
                        and 2 * max_slots * F * FEAT_BEST_BYTES <= p2p.cap // 2)
            # each pass's slab reduction runs the split scan of its slots right away
            # (reduce_split; N ranks: reduce_split_p2p); otherwise the level's
            # histograms are reduced, all-reduced and scanned in separate launches
            rs = comm is None or fuse_p2p
            fbest = self._buf("fbest", max_nodes * F * FEAT_BEST_BYTES // 8, torch.float64)
            # the level's finalisation buffers (needed by the reduce when it finalises)
            next_nodes = 2 * max_nodes
            part = self._buf("part", max_nodes * PART_INFO_BYTES // 4, torch.int32)
            nl = None
            if not last:
                nl = self._buf(f"link{nxt}", next_nodes * NODE_LINK_BYTES // 4, torch.int32)
                link[nxt] = nl
            nsplit = self._buf("nsplit", max_nodes * 9, torch.float64)  # NodeSplit = 72 B
            # one-pass levels of <= 64 nodes finalise in the last workgroup of their
            # reduce + split scan (LevelFin in csrc/tree_kernels.hip)
            fin = rs and max_nodes <= 64 and ((fuse_p2p and self.FUSE_FIN)
                                              or (comm is None and self.FUSE_FIN_LOCAL and plan["passes"] == 1))
            if fin and getattr(self, "_fin_ticket", None) is None:
                self._fin_ticket = torch.zeros((1,), dtype=torch.int32, device=self.dev)   # each launch leaves 0
            fin_args = (P(ctl_nxt), P(bm.edges), next_nodes, P(part), P(nl), P(self.tree_buf), self.capacity,
                        P(nsplit), P(self._fin_ticket if fin else None))

            def reduce(n_groups, wgpg, fg, slot_lo, slot_cnt):
                if rs and fuse_p2p:
                    if slot_lo != 0 or slot_cnt < max_slots:
                        raise RuntimeError("reduce_split_p2p: multi-pass level")   # excluded by fuse_p2p
                    ops.check(lib.h2omx_reduce_split_p2p(p2p.desc_ptr, P(partials), wgpg, fg, slot_cnt, P(full_prev),
                                                         P(full_cur), P(ctl_cur), P(link[cur]), P(bm.nvb),
                                                         P(tree_fmask), P(self.qscale), spp, nbt,
                                                         self.P2P_BLOCKS,
                                                         *(fin_args if fin else (None, None, 0, None, None, None, 0,
                                                                                 None, None)), st),
                              "reduce_split_p2p")
                    comm.stats["p2p_calls"] += 1
                    comm.stats["p2p_bytes"] += max_slots * self.per_node * 8
                elif rs and fin:
                    if slot_lo != 0 or slot_cnt < max_slots:
                        raise RuntimeError("reduce_split_fin: multi-pass level")   # excluded by fin
                    ops.check(lib.h2omx_reduce_split_fin(P(partials), wgpg, fg, slot_cnt, P(full_prev), P(full_cur),
                                                         P(ctl_cur), P(link[cur]), P(bm.nvb), P(tree_fmask),
                                                         P(self.qscale), spp, nbt, P(fbest), *fin_args, st),
                              "reduce_split_fin")
                elif rs:
                    ops.check(lib.h2omx_reduce_split(P(partials), wgpg, fg, slot_lo, slot_cnt, P(full_prev),
                                                     P(full_cur), P(ctl_cur), P(link[cur]), P(bm.nvb),
                                                     P(tree_fmask), P(self.qscale), spp, nbt, P(fbest), st),
                              "reduce_split")
                else:
                    ops.check(lib.h2omx_hist_reduce(P(partials), n_groups, wgpg, fg, F, nbt, slot_lo, slot_cnt,
                                                    P(ctl_cur), P(built), st), "hist_reduce")
            hist_elems = plan["slot_cnt"] * plan["fg"] * nbt
            partials = self._buf("partials", plan["n_groups"] * plan["wgpg"] * hist_elems, torch.int64)
            # level 0 streams every row; deeper levels touch only the built
            # (smaller) children -> wave-compacted kernel keeps atomics dense
            for ps in range(plan["passes"]):
                slot_lo = ps * plan["slot_cnt"]
                with T("hist"):
                    if d > 0 and fuse and self._fused_level(d):
                        # partition of level d - 1 fused in: nid_buf[d - 1] -> nid_buf[d]
                        ops.check(lib.h2omx_hist_build_route(
                            P(bm.codes), bm.npad, P(None if (d == 1 and self.implicit_root) else nid_buf[(d - 1) % 2]),
                            P(part_prev), P(ctl_nxt),
                            P(nid_buf[d % 2]), 1 if ps == 0 else 0, P(ctl_cur), P(bm.nvb), P(self.qscale), F, nbt,
                            plan["fg"], plan["n_groups"], plan["wgpg"], slot_lo, plan["slot_cnt"],
                            self.ROWS_PER_LANE, plan["threads"], P(self.pk),
                            (4 if self.pk32 else 2) + (64 if nid16 else 0),
                            P(partials), st),
                            "hist_build_route")
                    elif d == 0 and grad_fuse is not None:
                        gf = grad_fuse
                        ops.check(lib.h2omx_hist_build_grad(
                            P(bm.codes), bm.npad, P(ctl_cur), P(bm.nvb), P(self.qscale), tree_index & 0x7FFFFFFF,
                            F, nbt, plan["fg"], plan["n_groups"], plan["wgpg"], plan["slot_cnt"],
                            self.ROWS_PER_LANE, plan["threads"], P(self.pk), P(partials), P(gf["F"]), P(gf["y"]),
                            P(self.nid), P(self.tree_buf), self.capacity, P(g), P(h), 1 if gf["apply"] else 0,
                            0 if p.mode == 0 else 1, 0 if self.pk32 else 1, ctypes.addressof(gf["gp"]), st),
                            "hist_build_grad")
                    else:
                        # level 0 stores the packed quantised rows; deeper levels read them
                        # with the build slots the previous partition wrote
                        ops.check(lib.h2omx_hist_build(
                            P(bm.codes), bm.npad, P(g), P(s2),
                            P(None if (d == 0 and self.implicit_root) else (nid_buf[d % 2] if fuse else self.nid)),
                            P(link[cur]), P(ctl_cur), P(bm.nvb),
                            P(self.qscale), tree_index & 0x7FFFFFFF, F, nbt, plan["fg"], plan["n_groups"],
                            plan["wgpg"], slot_lo, plan["slot_cnt"], self.ROWS_PER_LANE, plan["threads"],
                            P(self.slot16), P(self.pk),
                            ((6 if pk_boost else 1 + (2 if self.pk32 else 0)) if d == 0
                             else 2 + (2 if self.pk32 else 0))
                            + ({8: 16, 4: 32}.get(self.L0_COPIES, 0) if l0_copies else 0),
                            P(partials), st),
                            "hist_build")
                with T("hist_reduce"):
                    reduce(plan["n_groups"], plan["wgpg"], plan["fg"], slot_lo, plan["slot_cnt"])
            if comm is not None and not fuse_p2p:
                with T("allreduce"):
                    comm.all_reduce_(built[: max_slots * self.per_node])
            with T("split"):
                if not rs:
                    ops.check(lib.h2omx_split_find(P(built), P(full_prev), P(full_cur), P(ctl_cur),
                                                   P(link[cur]), P(bm.nvb), P(tree_fmask), P(self.qscale), spp,
                                                   max_nodes, nbt, P(fbest), st), "split_find")
                if fin:
                    pass   # finalised inside the reduce launch
                elif fuse_p2p:
                    # waits for every rank's share of the split records (all-gathered
                    # into this rank's split table by reduce_split_p2p)
                    ops.check(lib.h2omx_node_best_finalize_p2p(p2p.desc_ptr, P(ctl_cur), P(ctl_nxt), spp, P(bm.edges),
                                                               P(bm.nvb), nbt, next_nodes, P(part), P(nl),
                                                               P(self.tree_buf), self.capacity, P(nsplit), st),
                              "node_best_finalize_p2p")
                else:
                    ops.check(lib.h2omx_level_finalize(P(fbest), P(ctl_cur), P(ctl_nxt), spp, P(bm.edges),
                                                       P(bm.nvb), nbt, next_nodes, P(part), P(nl),
                                                       P(self.tree_buf), self.capacity, P(nsplit), max_nodes,
                                                       self._lf_tiles(max_nodes),
                                                       st), "level_finalize")
            # leaves that can retire at this level: gids [base, base + n + n_next)
            win = min(3 * max_nodes, self.capacity)
            with T("partition"):
                if fuse and last:
                    rg = self.regrad if (chain and w is None) else None   # (F, y, GradParams)
                    # chained graph steps: int16 leaf ids into the free node-id buffer
                    # for boost_update; otherwise int32 into self.nid
                    leaf16 = chain and nid16
                    self.leaf16_buf = nid_buf[(d + 1) % 2] if leaf16 else None
                    ops.check(lib.h2omx_partition_final(P(bm.codes), bm.npad, P(nid_buf[d % 2]),
                                                        P(self.leaf16_buf if leaf16 else self.nid),
                                                        P(part), nbt, P(g), P(h), P(w), P(self.qscale),
                                                        self.capacity, P(self.leaf_acc), P(ctl_cur), P(ctl_nxt),
                                                        self.part_blocks, P(rg[0] if rg else None),
                                                        P(rg[1] if rg else None),
                                                        ctypes.addressof(rg[2]) if rg else None,
                                                        (3 if leaf16 else 1) if nid16 else 0,
                                                        P(rg[3] if rg else None), st),
                              "partition_final")
                elif fuse and not self._fused_level(d + 1):
                    ops.check(lib.h2omx_partition_route(P(bm.codes), bm.npad, P(nid_buf[d % 2]),
                                                        P(nid_buf[(d + 1) % 2]), P(part), nbt, P(ctl_cur),
                                                        P(ctl_nxt), self.part_blocks, P(self.slot16),
                                                        3 if nid16 else 0, st),
                              "partition_route")
                elif not fuse:
                    ops.check(lib.h2omx_partition(P(bm.codes), bm.npad, P(self.nid), P(part), nbt, P(g), P(h),
                                                  P(w), P(self.qscale), self.capacity, P(self.leaf_acc),
                                                  P(ctl_cur), P(ctl_nxt), win, self.part_blocks, 1 if last else 0,
                                                  P(None if last else self.slot16), st),
                              "partition")
            part_prev = part
            full_prev = full_cur
            max_nodes = next_nodes
        # exact leaf values (sums accumulated by the partition kernels); N ranks over
        # P2P exchange the sums inside the leaf finalisation
        leaf_p2p = p2p is not None and self.gbound is None and self.capacity * 3 * 8 * p2p.world <= p2p.cap
        if comm is not None and not leaf_p2p:
            with T("allreduce"):
                comm.all_reduce_(self.leaf_acc)
        with T("leaf"):
            if leaf_p2p:
                ops.check(lib.h2omx_leaf_finalize_p2p(p2p.desc_ptr, P(self.leaf_acc), P(final_ctl), P(self.qscale),
                                                      spp, P(self.tree_buf), self.capacity, 1 if chain else 0,
                                                      P(smax if chain else None), p.mode,
                                                      self.max_rows_per_wg if chain else 0,
                                                      P(self.ctl[0] if chain else None),
                                                      P(link[0] if chain else None), self.row_base,
                                                      P(self.tree_ctr if chain else None), st), "leaf_finalize_p2p")
                comm.stats["p2p_calls"] += 1
                comm.stats["p2p_bytes"] += self.capacity * 3 * 8
            elif chain:
                ops.check(lib.h2omx_leaf_finalize_begin(P(self.leaf_acc), P(final_ctl), P(self.qscale), spp,
                                                        P(self.tree_buf), self.capacity, P(smax), p.mode,
                                                        self.max_rows_per_wg, P(self.ctl[0]), P(link[0]),
                                                        self.row_base, P(self.tree_ctr), st), "leaf_finalize_begin")
            else:
                self._leaf_finalize(final_ctl, spp, st)
        self._final_ctl = final_ctl
        return self.tree_buf

    def can_chain(self, fixed: bool) -> bool:
        """Graph replay may fold tree_begin into the previous tree's leaf
        finalisation: fixed gradient bounds (the scales do not depend on the
        boost pass that runs in between), the scan engine, the plain leaf pass
        (no monotone Newton re-derivation) and a device tree counter."""
        return (fixed and not self.segmented and self.gbound is None and self.tree_ctr is not None
                and self.CHAIN_BEGIN)

    # chained graph steps: boost_update also writes the next tree's 16-bit packed
    # level-0 rows, so level 0 reads 4 bytes per row and feature group instead of
    # (g, s2) = 8 bytes (4 groups at level 0: ~220 MB less traffic at 11M rows)
    pk_in_boost = False
    # chained graph steps of unweighted rows: boost_update stores no (g, h); the
    # final partition re-derives them from (margins, labels, GradParams, byte labels)
    regrad = None
    leaf16_buf = None   # int16 leaf ids of the last chained tree (boost_update reads them)

    def can_pack_in_boost(self) -> bool:
        return (self.pk32 and self.implicit_root and not self.segmented
                and self.L0_COPIES in (1, 4, 8))

    def begin(self, smax: torch.Tensor, tree_index: int) -> None:
        """tree_begin: fixed-point scales, level-0 control block / root link,
        zeroed leaf sums (and, with a device tree counter, its advance)."""
        P = ops.P
        ops.check(self.lib.h2omx_tree_begin(P(smax), self.p.mode, self.max_rows_per_wg, P(self.qscale),
                                            P(self.ctl[0]), P(self._buf("link0", 4, torch.int32)),
                                            P(self.leaf_acc), self.leaf_acc.numel(), self.row_base,
                                            tree_index & 0x7FFFFFFF, P(self.tree_ctr), ops.stream(self.dev)),
                  "tree_begin")

    # data-parallel direct levels: histogram chunk all-reduced per call (bytes)
    DIRECT_DP_CHUNK_BYTES = 64 << 20

    def _direct_dp(self, comm, idx_in, gs, seg_start, seg_cnt, ctl_cur, tree_fmask, spp, max_nodes, nsplit, st):
        """Direct level over N row shards: per node chunk, this rank's eligible-
        feature histograms (h2omx_direct_dp phase 0) -> all-reduce -> the scan
        (phase 1) writes the nodes' NodeSplit records, identical on every rank."""
        lib, P, bm = self.lib, ops.P, self.bm
        stride = int(lib.h2omx_direct_dp_stride(spp, self.nbt))
        chunk = max(1, min(max_nodes, self.DIRECT_DP_CHUNK_BYTES // (8 * stride)))
        dh = self._buf("direct_dp", chunk * stride, torch.int64)
        for node0 in range(0, max_nodes, chunk):
            nc = min(chunk, max_nodes - node0)
            for phase in (0, 1):
                ops.check(lib.h2omx_direct_dp(phase, P(self.codes_rm), bm.fp, P(idx_in), P(gs["g"]), P(gs["s"]),
                                              P(seg_start), P(seg_cnt), P(ctl_cur), P(bm.nvb), P(tree_fmask),
                                              P(self.qscale), spp, self.nbt, node0, nc, P(dh), P(nsplit),
                                              gs["pos"], None, st), "direct_dp")
                if phase == 0:
                    comm.all_reduce_(dh[: nc * stride])
        self.stats["direct_dp_levels"] = self.stats.get("direct_dp_levels", 0) + 1

    # node counts of levels above SYNC_NODE_CAP read back early: a pinned copy of
    # the next level's (nodes, slots) + event right after its finalisation, so
    # the host waits for the finalisation only while the level's partition
    # kernels still run (instead of draining the stream at the next level's top)
    _ctl_host = None

    def _count_ahead(self, ctl_nxt: torch.Tensor, parity: int) -> None:
        if self._ctl_host is None:
            self._ctl_host = torch.empty((2, 2), dtype=torch.int32, pin_memory=True)
            self._ctl_ev = [torch.cuda.Event(), torch.cuda.Event()]
            self._ctl_pending = [False, False]
        self._ctl_host[parity].copy_(ctl_nxt[:2], non_blocking=True)
        self._ctl_ev[parity].record()
        self._ctl_pending[parity] = True

    def _count_now(self, ctl_cur: torch.Tensor, parity: int) -> tuple[int, int]:
        self.stats["host_syncs"] += 1
        if self._ctl_host is not None and self._ctl_pending[parity]:
            self._ctl_ev[parity].synchronize()
            self._ctl_pending[parity] = False
            return int(self._ctl_host[parity, 0]), int(self._ctl_host[parity, 1])
        n_now, s_now = [int(v) for v in ctl_cur[:2].tolist()]
        return n_now, s_now

    def _build_seg(self, g, h, w, tree_index, tree_fmask, smax, fixed):
        """Row-partitioned level pipeline (csrc/tree_kernels.hip, "segmented"
        section): each level reads only the rows of the nodes it builds."""
        lib, bm, p = self.lib, self.bm, self.p
        st = ops.stream(self.dev)
        P = ops.P
        F, nbt, n = self.F, self.nbt, bm.n
        spp = self._params(tree_index)
        sp = self._sp
        comm = self.comm if (self.comm is not None and self.comm.world_size > 1) else None
        if comm is not None and not fixed:
            comm.all_reduce_(smax, "max")
        s2 = w if p.mode == 0 else h
        B = self._buf
        i32 = torch.int32
        link = [B("link0", 4, i32), None]
        seg = [[B(f"seg_start{k}", 2, i32), B(f"seg_cnt{k}", 2, i32), B(f"hc_first{k}", 3, i32),
                B(f"pc_first{k}", 3, i32), B(f"slot_node{k}", 2, i32)] for k in (0, 1)]
        built = B("built", self.per_node, torch.int64)
        ops.check(lib.h2omx_tree_begin_seg(P(smax), p.mode, self.max_rows_per_wg, P(self.qscale),
                                           P(self.ctl[0]), P(link[0]), P(self.leaf_acc), self.leaf_acc.numel(),
                                           P(built), self.per_node, n, self.hc_rows, P(seg[0][0]), P(seg[0][1]),
                                           P(seg[0][2]), P(seg[0][3]), P(seg[0][4]), self.row_base,
                                           tree_index & 0x7FFFFFFF, P(self.tree_ctr), st),
                  "tree_begin_seg")
        full_prev = None
        max_depth = p.max_depth
        final_ctl = self.ctl[max_depth % 2]
        max_nodes = 1
        built_zeroed = True          # tree_begin_seg zeroed level 0's histogram
        hc_cap = -(-n // self.hc_rows)
        pc_cap = -(-n // self.pc_rows)
        idx_in = None
        # (g, s2) as the current level reads them: by row at level 0, afterwards in segment order
        # (part_scatter moves them with the rows, so the histogram passes read them contiguously)
        gs = {"g": g, "s": s2, "pos": 0}
        # bagged trees: the root segment holds only the rows of nonzero weight, (g, s2) already
        # in its order; the others get their leaf from the finished tree (bag_route_out)
        bagged = (self.BAG_COMPACT and self.bag_compact and w is not None and s2 is not None and comm is None
                  and self.catf is None and n > 0)
        if bagged:
            gs = {"g": B("bag_g", n + 64, torch.float32), "s": B("bag_s", n + 64, torch.float32), "pos": 1}
            idx_in = B("bag_idx", n + 64, i32)
            ops.check(lib.h2omx_bag_compact(P(w), n, P(g), P(s2), P(B("bag_cnt", -(-n // 4096) + 1, i32)),
                                            P(idx_in), P(gs["g"]), P(gs["s"]), P(seg[0][1]), P(seg[0][2]),
                                            P(seg[0][3]), self.hc_rows, st), "bag_compact")
        # mean leaves (DRF) read no H sum: the retiring rows skip their random h[r] gather
        mean_leaves = p.leaf_mode == 1 and self.MEAN_LEAVES_NO_H

        def route(d, last, max_nodes, next_nodes, part, nl, seg_start, seg_cnt, pc_first, ctl_cur, ctl_nxt,
                  idx_in, next_direct, ec=None, cpos=(None, None)):
            """part_count -> level_close -> part_scatter: rows into their next-level segments.
            ec: (codes, stride, nodeq) of the direct pass - split codes read in segment order.
            cpos: (in, out) column-major plane positions moved with the rows (COLMAJOR_EVERY)."""
            cur, nxt = d % 2, (d + 1) % 2
            nbuilt = None
            max_pc = pc_cap + max_nodes
            pwave = int(max_nodes >= self.PART_WAVE_NODES or ec is not None)
            ecodes, ecs, nodeq = ec if ec is not None else (None, 0, None)
            # row directions stored by part_count for part_scatter (not on the last level: no count pass)
            dirb = B("dirb", n + 64, torch.int8) if not last else None
            pc_left = B("pc_left", max_pc, i32)
            node_nl = B("node_nl", 2 * max_nodes, i32)
            idx_out = None
            write_nid = 0
            if not last:
                nstart, ncnt, nhc, npc, nslot = seg[nxt]
                nstart = seg[nxt][0] = B(f"seg_start{nxt}", next_nodes, i32)
                ncnt = seg[nxt][1] = B(f"seg_cnt{nxt}", next_nodes, i32)
                nhc = seg[nxt][2] = B(f"hc_first{nxt}", next_nodes + 1, i32)
                npc = seg[nxt][3] = B(f"pc_first{nxt}", next_nodes + 1, i32)
                nslot = seg[nxt][4] = B(f"slot_node{nxt}", max(1, max_nodes), i32)
                next_seg_hist = (not next_direct) and (max_nodes > self.SCAN_SLOTS or next_nodes > self.SYNC_NODE_CAP)
                # live-row node ids feed the next level's scan histograms only
                write_nid = 0 if (next_seg_hist or next_direct) else 1
                nbuilt = None
                if next_seg_hist:
                    nbuilt = B("built", max_nodes * self.per_node, torch.int64)
                ops.check(lib.h2omx_part_count(P(bm.codes), bm.npad, P(idx_in), P(seg_start), P(seg_cnt),
                                               P(pc_first), P(ctl_cur), P(part), nbt, max_pc, P(pc_left), pwave,
                                               P(dirb), P(ecodes), ecs, P(nodeq), None, bm.fp, None, st),
                          "part_count")
                if max_nodes <= self.CLOSE_SINGLE_BLOCK:
                    ops.check(lib.h2omx_level_close(P(ctl_cur), P(ctl_nxt), P(part), P(nl), P(seg_start),
                                                    P(seg_cnt), P(pc_first), P(pc_left), P(node_nl), P(nstart),
                                                    P(ncnt), P(nhc), P(npc), P(nslot), self.hc_rows, P(nbuilt),
                                                    self.per_node, st), "level_close")
                else:
                    pc_excl = B("pc_excl", max_pc, i32)
                    tiles = B("scan_tiles", max(max_pc, next_nodes) // 1024 + 2, i32)
                    cnt_h = B("cnt_h", next_nodes, i32)
                    cnt_p = B("cnt_p", next_nodes, i32)
                    aux = B("close_aux", 4, i32)
                    ops.check(lib.h2omx_level_close_mb(P(ctl_cur), P(ctl_nxt), P(part), P(nl), P(seg_start),
                                                       P(seg_cnt), P(pc_first), P(pc_left), P(node_nl), P(nstart),
                                                       P(ncnt), P(nhc), P(npc), P(nslot), self.hc_rows, P(nbuilt),
                                                       self.per_node, max_nodes, max_pc, P(pc_excl), P(tiles),
                                                       P(cnt_h), P(cnt_p), P(aux), st), "level_close_mb")
                idx_out = self.idx[d % 2]
            gout = sout = None
            # last level: leaf sums read (g, s2) in segment order where the previous
            # scatter left them
            segf = 0
            if last and pwave and gs["pos"] == 1:
                segf = 2 | (4 if p.mode != 0 else 0)
            if not last and self.PERMUTE_GS:
                gout = B(f"gperm{d % 2}", n + 64, torch.float32)
                sout = None if s2 is None else B(f"sperm{d % 2}", n + 64, torch.float32)
            ops.check(lib.h2omx_part_scatter(P(bm.codes), bm.npad, P(idx_in), P(idx_out), P(self.nid), write_nid,
                                             P(seg_start), P(seg_cnt), P(pc_first), P(pc_left), P(node_nl),
                                             P(ctl_cur), P(part), nbt, P(g), P(None if mean_leaves else h), P(w),
                                             P(self.qscale),
                                             self.capacity, P(self.leaf_acc), max_pc, pwave | segf, P(dirb), P(gs["g"]),
                                             P(gs["s"]), P(gout), P(sout), P(ecodes), ecs, P(nodeq),
                                             P(self.codes_rm), None, None, bm.fp, P(cpos[0]),
                                             P(None if last else cpos[1]), st),
                      "part_scatter")
            if gout is not None:
                gs.update(g=gout, s=sout, pos=1)
            else:
                gs.update(g=g, s=s2, pos=0)
            return idx_out, nbuilt is not None

        direct = False
        # direct mode pays n x (eligible features) per level; the subtraction path
        # n / 2 x F + nodes x F x bins: direct only for few eligible features (DRF mtries)
        exp_elig = min(p.mtries, F) if p.mtries > 0 else F * min(1.0, p.col_sample_rate)
        # (N ranks: the direct histograms of a node chunk are all-reduced between
        # the build and the scan, h2omx_direct_dp)
        direct_ok = (self.DIRECT_MIN_NODES > 0 and F <= 1024
                     and exp_elig <= self.DIRECT_MAX_ELIG and self.catf is None)
        # column-major planes (COLMAJOR_EVERY): level of the last transpose, positions of the next level
        cm_last, cm_pos = None, None
        if self._ctl_host is not None:
            self._ctl_pending = [False, False]    # (a tree that ended early left one unread)
        for d in range(max_depth):
            cur, nxt = d % 2, (d + 1) % 2
            ctl_cur, ctl_nxt = self.ctl[cur], self.ctl[nxt]
            if max_nodes > self.SYNC_NODE_CAP:
                n_now, s_now = self._count_now(ctl_cur, cur)
                if n_now == 0:
                    final_ctl = ctl_cur     # tree finished early: ctl_cur holds its final TOTAL
                    break
                max_nodes, max_slots = n_now, s_now
            else:
                max_slots = 1 if d == 0 else max(1, max_nodes // 2)
            last = d == max_depth - 1
            seg_start, seg_cnt, hc_first, pc_first, slot_node = seg[cur]
            direct = direct or (direct_ok and d > 0 and max_nodes >= self.DIRECT_MIN_NODES)
            if direct:
                # eligible-feature histograms of every node built and scanned in LDS
                sp.depth = d
                sp.children_leaves = 1 if last else 0
                next_nodes = 2 * max_nodes
                nsplit = B("nsplit", max_nodes * 9, torch.float64)
                part = B("part", max_nodes * PART_INFO_BYTES // 4, i32)
                nl = None
                if not last:
                    nl = B(f"link{nxt}", next_nodes * NODE_LINK_BYTES // 4, i32)
                    link[nxt] = nl
                # one wave per node for small nodes, one workgroup per row chunk while nodes
                # are large (big nodes spread over many workgroups), else one workgroup per node
                max_pc = pc_cap + max_nodes
                n_elig = min(p.mtries, F) if p.mtries > 0 else F
                slab = tot_slab = ticket = None
                if n < self.DIRECT_WAVE_ROWS * max_nodes and F <= 256:
                    dmode = 1
                elif self.DIRECT_CHUNKED and n_elig * nbt * 16 <= 65536:
                    dmode = 2
                    slab = B("dslab", max_pc * n_elig * nbt, torch.int64)
                    tot_slab = B("dtot", 2 * max_pc, torch.int64)
                    ticket = self._ticket_buf(max_nodes)
                else:
                    dmode = 0
                ec = None
                # every eligible feature in one LDS batch (batch sizes of h2omx_seg_direct;
                # wave mode: packed nodes - all but those of >= 64K rows - hold twice the
                # features per batch, and a node scanned in several batches stores no
                # eligible codes: the partition reads its code rows instead)
                one_batch = ({0: 98304, 1: 8192, 2: 1 << 30}[dmode] // (16 * nbt)) * (2 if dmode == 1 else 1) >= n_elig
                if self.ECODES and n_elig <= 16 and one_batch:
                    ecs = 8 if n_elig <= 8 else 16
                    ec = (B("ecodes", (n + 64) * ecs, torch.uint8), ecs, B("nodeq", max_nodes, i32))
                ecodes, ecs, nodeq = ec if ec is not None else (None, 0, None)
                ccol = cpos_cur = cpos_next = None
                plane = 0
                if comm is not None:
                    self._direct_dp(comm, idx_in, gs, seg_start, seg_cnt, ctl_cur, tree_fmask, spp, max_nodes,
                                    nsplit, st)
                    ec = None
                else:
                    # (the transpose stages 256 code rows in LDS: rows of <= 384 bytes)
                    if self.COLMAJOR_EVERY > 0 and dmode == 2 and bm.fp <= 384:
                        plane = -(-n // 256) * 256
                        ccol = B("ccol", F * plane, torch.uint8)
                        if cm_pos is None or d - cm_last >= self.COLMAJOR_EVERY:
                            ops.check(lib.h2omx_seg_colmajor(P(self.codes_rm), bm.fp, F, P(idx_in), n, bm.npad,
                                                             P(ccol), plane, st), "seg_colmajor")
                            cm_last = d
                        else:
                            cpos_cur = cm_pos
                    # positions for the next level only if it is surely a row-chunk level too
                    cm_pos = None
                    if ccol is not None and not last and n >= self.DIRECT_WAVE_ROWS * next_nodes:
                        cpos_next = cm_pos = B(f"cpos{nxt}", n + 64, i32)
                    ops.check(lib.h2omx_seg_direct(P(self.codes_rm), bm.fp,
                                                   P(idx_in), P(gs["g"]), P(gs["s"]),
                                                   P(seg_start), P(seg_cnt), P(ctl_cur), P(bm.nvb), P(tree_fmask),
                                                   P(self.qscale), tree_index & 0x7FFFFFFF, spp, nbt, max_nodes,
                                                   dmode, P(pc_first), max_pc, P(slab), P(tot_slab), P(ticket),
                                                   P(nsplit), gs["pos"], P(ecodes), ecs, P(nodeq), P(ccol),
                                                   P(cpos_cur), plane, st),
                              "seg_direct")
                ops.check(lib.h2omx_level_finalize_ns(P(nsplit), P(ctl_cur), P(ctl_nxt), spp, P(bm.edges),
                                                      P(bm.nvb), nbt, next_nodes, P(part), P(nl), P(self.tree_buf),
                                                      self.capacity, max_nodes,
                                                      self._lf_tiles(max_nodes), st),
                          "level_finalize_ns")
                if not last and next_nodes > self.SYNC_NODE_CAP:
                    self._count_ahead(ctl_nxt, nxt)
                idx_in, _ = route(d, last, max_nodes, next_nodes, part, nl, seg_start, seg_cnt, pc_first, ctl_cur,
                                  ctl_nxt, idx_in, True, ec, (cpos_cur, cpos_next))
                full_prev = None
                max_nodes = next_nodes
                continue
            seg_hist = max_slots > self.SCAN_SLOTS or max_nodes > self.SYNC_NODE_CAP
            built = B("built", max_slots * self.per_node, torch.int64)
            if seg_hist and not built_zeroed:
                built[: max_slots * self.per_node].zero_()
            built_zeroed = False
            if seg_hist:
                max_hc = hc_cap + max_slots
                slab = B("seg_slab", max_hc * self.seg_groups * self.seg_fg * nbt, torch.int64)
                ops.check(lib.h2omx_hist_build_seg(P(self.codes_rm), bm.fp, P(idx_in), P(gs["g"]), P(gs["s"]),
                                                   P(seg_start), P(seg_cnt), P(hc_first), P(ctl_cur), P(bm.nvb),
                                                   P(self.qscale), tree_index & 0x7FFFFFFF, F, nbt, self.seg_fg,
                                                   self.seg_groups, self.hc_rows, max_hc, self.seg_threads, P(slab),
                                                   gs["pos"], None, None, st), "hist_build_seg")
                ksplit = max(1, min(32, 4096 // max(1, max_slots * ((F * nbt + 255) // 256))))
                ksplit = max(ksplit, 4)
                ops.check(lib.h2omx_hist_reduce_seg(P(slab), P(hc_first), P(slot_node), P(ctl_cur), F, nbt,
                                                    self.seg_fg, self.seg_groups, max_slots, ksplit, P(built), st),
                          "hist_reduce_seg")
            else:
                plan = self.plan_level(max_slots)
                hist_elems = plan["slot_cnt"] * plan["fg"] * nbt
                partials = B("partials", plan["n_groups"] * plan["wgpg"] * hist_elems, torch.int64)
                for ps in range(plan["passes"]):
                    slot_lo = ps * plan["slot_cnt"]
                    ops.check(lib.h2omx_hist_build(P(bm.codes), bm.npad, P(g), P(s2), P(self.nid), P(link[cur]),
                                                   P(ctl_cur), P(bm.nvb), P(self.qscale), tree_index & 0x7FFFFFFF,
                                                   F, nbt, plan["fg"], plan["n_groups"], plan["wgpg"], slot_lo,
                                                   plan["slot_cnt"], self.ROWS_PER_LANE, plan["threads"],
                                                   None, None, 0, P(partials), st), "hist_build")
                    ops.check(lib.h2omx_hist_reduce(P(partials), plan["n_groups"], plan["wgpg"], plan["fg"], F, nbt,
                                                    slot_lo, plan["slot_cnt"], P(ctl_cur), P(built), st),
                              "hist_reduce")
            if comm is not None:
                comm.all_reduce_(built[: max_slots * self.per_node])
            full_cur = None if last else B(f"full{cur}", max_nodes * self.per_node, torch.int64)
            fbest = B("fbest", max_nodes * F * FEAT_BEST_BYTES // 8, torch.float64)
            self._cat_level(max_nodes)
            sp.depth = d
            sp.children_leaves = 1 if last else 0
            ops.check(lib.h2omx_split_find(P(built), P(full_prev), P(full_cur), P(ctl_cur), P(link[cur]),
                                           P(bm.nvb), P(tree_fmask), P(self.qscale), spp, max_nodes, nbt,
                                           P(fbest), st), "split_find")
            next_nodes = 2 * max_nodes
            part = B("part", max_nodes * PART_INFO_BYTES // 4, i32)
            nl = None
            if not last:
                nl = B(f"link{nxt}", next_nodes * NODE_LINK_BYTES // 4, i32)
                link[nxt] = nl
            nsplit = B("nsplit", max_nodes * 9, torch.float64)
            ops.check(lib.h2omx_level_finalize(P(fbest), P(ctl_cur), P(ctl_nxt), spp, P(bm.edges), P(bm.nvb), nbt,
                                               next_nodes, P(part), P(nl), P(self.tree_buf), self.capacity,
                                               P(nsplit), max_nodes, self._lf_tiles(max_nodes), st),
                      "level_finalize")
            if not last and next_nodes > self.SYNC_NODE_CAP:
                self._count_ahead(ctl_nxt, nxt)
            idx_in, built_zeroed = route(d, last, max_nodes, next_nodes, part, nl, seg_start, seg_cnt, pc_first,
                                         ctl_cur, ctl_nxt, idx_in, False)
            full_prev = full_cur
            max_nodes = next_nodes
        if bagged:
            ops.check(lib.h2omx_bag_route_out(P(w), n, P(self.codes_rm), bm.fp, P(self.tree_buf), nbt,
                                              P(self.nid), st),
                      "bag_route_out")
        if comm is not None:
            comm.all_reduce_(self.leaf_acc)
        self._leaf_finalize(final_ctl, spp, st)
        self._final_ctl = final_ctl
        return self.tree_buf

    def _leaf_finalize(self, final_ctl, spp, st):
        """Leaf values from the exact leaf sums.  Monotone constraints with
        squared-error splits and Newton leaves (GBM, mode 0 / leaf_mode 0): the
        node intervals are re-derived on the Newton (-G/H) scale of the leaf
        values (mono_newton_kernel) instead of the -G/W scale the level
        finalisation could use (the histograms carry W, not H)."""
        lib, P, p = self.lib, ops.P, self.p
        if self.gbound is not None and p.mode == 0 and p.leaf_mode == 0:
            cap = self.capacity
            scratch = self._buf("mono_scratch", ((cap * 4 + 15) // 16) * 16 + cap * 32, torch.uint8)
            ops.check(lib.h2omx_leaf_finalize_mono(P(self.leaf_acc), P(final_ctl), P(self.qscale), spp,
                                                   P(self.tree_buf), cap, P(scratch), st), "leaf_finalize_mono")
        else:
            ops.check(lib.h2omx_leaf_finalize(P(self.leaf_acc), P(final_ctl), P(self.qscale), spp,
                                              P(self.tree_buf), self.capacity, st), "leaf_finalize")

    def reduce_stats(self) -> None:
        """Fold the per-block maxima written by the gradient kernels into stat_max."""
        ops.check(self.lib.h2omx_stat_reduce(ops.P(self.stat_slab), ops.P(self.stat_max), ops.stream(self.dev)),
                  "stat_reduce")

    def tree_size(self) -> torch.Tensor:
        """Device scalar with the node count of the last tree (ctl TOTAL)."""
        return self._final_ctl[3]


def per_slot_fits(F: int, nbt: int, threads: int) -> bool:
    """One slot of F x nbt packed histograms + the entry stages fit 160 KB LDS."""
    return F * nbt * 8 + (threads // 64) * 2048 <= 160 * 1024


def global_rows(n: int, comm) -> tuple[int, int]:
    """(global index of this rank's first row, global row count)."""
    if comm is None or comm.world_size <= 1:
        return 0, n
    counts = comm.all_gather_cat(torch.tensor([n], dtype=torch.int64, device=comm.device)).cpu().tolist()
    return int(sum(counts[: comm.rank])), int(sum(counts))


def global_row_base(n: int, comm) -> int:
    return global_rows(n, comm)[0]


def trees_from_bytes(buf: np.ndarray, capacity: int) -> np.ndarray:
    """View raw bytes as [ntrees][capacity] TREE_NODE_DTYPE records (a view of
    the downloaded buffer, no copy: a 10-tree DRF depth-20 forest is ~400 MB,
    and the former tobytes() copy cost ~30 ms a fit)."""
    if buf.ndim == 2 and buf.dtype == np.uint8 and buf.shape[1] == capacity * TREE_NODE_DTYPE.itemsize \
            and buf.strides[1] == 1:
        return buf.view(TREE_NODE_DTYPE)   # rows of a larger host array (async download): no copy either
    return np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1).view(TREE_NODE_DTYPE).reshape(-1, capacity)


# fixed (max|g|, max h, max w) of unweighted rows per distribution: a tree whose
# level 0 computes the gradients itself quantises with these (can_fuse_grad)
GRAD_BOUNDS = {"bernoulli": (1.0, 0.25, 1.0), "laplace": (1.0, 1.0, 1.0), "quantile": (1.0, 1.0, 1.0)}


def grad_bounds_tensor(dist: str, device) -> torch.Tensor:
    """stat_max image (float bits as int32) of GRAD_BOUNDS[dist]"""
    b = np.array(list(GRAD_BOUNDS[dist]) + [0.0], np.float32).view(np.int32)
    return torch.from_numpy(b.copy()).to(device)


def make_grad_params(dist: str, apply_tree: bool, sample_rate: float, seed: int, tree_index: int,
                     tweedie_power: float = 1.5, quantile_alpha: float = 0.5, huber_delta: float = 1.0,
                     row_base: int = 0) -> GradParams:
    from .structs import DIST_CODES

    gp = GradParams()
    gp.dist = DIST_CODES[dist]
    gp.apply_tree = 1 if apply_tree else 0
    gp.sample_rate = sample_rate
    gp.seed = seed & 0xFFFFFFFF
    gp.tree_index = tree_index
    gp.tweedie_power, gp.quantile_alpha, gp.huber_delta = tweedie_power, quantile_alpha, huber_delta
    gp.row_base = row_base
    return gp
