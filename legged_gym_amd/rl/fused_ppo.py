"""The PPO update of rsl_rl v1.0.x (`PPO.update`; legged_robot_config.py:226-239) as an explicit
forward/backward over flat parameter/gradient buffers — no autograd graph, no per-op launches.

Per minibatch (M rows), on one stream, no host synchronisation:
  weight preparation (lgx_copy2d: zero-padded layer-1 weights, transposed hidden weights) on the
  first minibatch of an update; afterwards the Adam step writes these copies (lgx_adam_clip_mirror)
  gather obs rows (lgx_ppo_gather_rows_padded, K padded to a multiple of 16)
  hidden layers: lgx_gemm_nt with the bias + ELU epilogue, {actor, critic} batched in one launch
                 (LGX_PPO_GEMM=auto: library GEMM + lgx_bias_act for layers 2..L)
  heads + loss: lgx_ppo_loss = output layers (in-kernel dot products), log-prob / ratio / clipped surrogate / clipped value loss / entropy
         / KL and the analytic gradient w.r.t. mu, value, std, head biases; its finalize applies the
         device-side adaptive schedule (data-parallel: lgx_ppo_adapt_lr after the gradient
         all-reduce the KL rides in)
  backward: lgx_head_bwd, then per layer split-K bmm for dW, lgx_gemm_nt for dA with the ELU'
            + bias-gradient column-sum epilogue
  (hidden widths that are not multiples of 128, or LGX_PPO_GEMM=lib: library GEMMs through torch
   + lgx_bias_act / lgx_elu_bwd_colsum instead of lgx_gemm_nt)
  lgx_reduce_slices: all split-K and bias partials -> flat gradient (one launch)
  [ONE all-reduce over RCCL when data-parallel: flat gradient + the minibatch KL]
  lgx_adam_clip[_mirror]: clip_grad_norm_(max_grad_norm) + Adam on the flat buffers (+ the GEMM weight copies)
The module's nn.Parameters become views of the flat buffer, so state_dict / load_state_dict /
the rollout's fused inference see the updated weights; the optimizer is `FlatAdam`, whose
state_dict has torch.optim.Adam's format (checkpoints stay loadable by upstream tooling).
"""
import ctypes as C
import os
import time

import torch
import torch.nn as nn

from legged_gym_amd.sim import abi


class _TunedGemms:
    """The GEMM solution table tuned on MI355X for the PPO-update shapes (torch TunableOp,
    rocBLAS / hipBLASLt solutions; regenerate with tools/tune_gemms.sh), scoped: TunableOp is
    switched on, read-only (no tuning, no recording of untuned shapes), with this table's file
    name, only inside `with` blocks around the update's library GEMMs; every TunableOp setting
    the caller had (enable, tuning, recording, file name) is restored on exit, so other torch GEMMs
    of the process are unaffected.  Shapes not in the table run the library default.
    LGX_TUNED_GEMMS=0 disables."""
    _loaded = None

    def __init__(self):
        self.ok = False
        if os.environ.get("LGX_TUNED_GEMMS", "1") == "0":
            return
        import torch.cuda.tunable as tunable
        from legged_gym_amd import LEGGED_GYM_ROOT_DIR
        path = os.path.join(LEGGED_GYM_ROOT_DIR, "resources", "tunableop", "ppo_gemms_gfx950.csv")
        if not os.path.exists(path):
            return
        self.tunable, self.path = tunable, path
        if _TunedGemms._loaded is None:
            saved = self._save()
            self._apply()
            _TunedGemms._loaded = bool(tunable.read_file(path))
            self._restore(saved)
        self.ok = _TunedGemms._loaded

    def _save(self):
        t = self.tunable
        return (t.is_enabled(), t.tuning_is_enabled(), t.record_untuned_is_enabled(), t.get_filename())

    def _apply(self):
        t = self.tunable
        t.enable(True)
        t.tuning_enable(False)
        t.record_untuned_enable(False)
        t.set_filename(self.path, insert_device_ordinal=False)

    def _restore(self, saved):
        t = self.tunable
        enabled, tuning, record, filename = saved
        t.tuning_enable(tuning)
        t.record_untuned_enable(record)
        if filename:
            t.set_filename(filename, insert_device_ordinal=False)
        t.enable(enabled)

    def __enter__(self):
        if self.ok:
            self.saved = self._save()
            self._apply()
        return self

    def __exit__(self, *exc):
        if self.ok:
            self._restore(self.saved)
        return False


def _vp(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class FlatAdam:
    """torch.optim.Adam (no weight decay, no amsgrad) over one flat parameter buffer, with the
    learning rate and the step counter resident on the device."""

    def __init__(self, params, flat_p, flat_g, lr, betas=(0.9, 0.999), eps=1e-8):
        self.params = list(params)
        self.flat_p, self.flat_g = flat_p, flat_g
        self.m = torch.zeros_like(flat_p)
        self.v = torch.zeros_like(flat_p)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=flat_p.device)
        self.lr_dev = torch.full((1,), float(lr), dtype=torch.float64, device=flat_p.device)
        self.betas, self.eps = betas, eps
        self.param_groups = [dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False, maximize=False,
                                  foreach=None, capturable=False, differentiable=False, fused=None)]

    def _views(self, buf):
        base = self.flat_p.data_ptr()
        out = []
        for p in self.params:
            off = (p.data_ptr() - base) // 4
            out.append(buf[off:off + p.numel()].view_as(p))
        return out

    def zero_grad(self, set_to_none=False):
        self.flat_g.zero_()

    def state_dict(self):
        step = float(self.step_dev.item())
        ms, vs = self._views(self.m), self._views(self.v)
        state = {i: {"step": torch.tensor(step), "exp_avg": ms[i].clone(), "exp_avg_sq": vs[i].clone()}
                 for i in range(len(self.params)) if step > 0}
        g = dict(self.param_groups[0])
        g["lr"] = float(self.lr_dev.item())
        g["params"] = list(range(len(self.params)))
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, d):
        g = d["param_groups"][0]
        self.lr_dev.fill_(float(g["lr"]))
        self.param_groups[0]["lr"] = float(g["lr"])
        ms, vs = self._views(self.m), self._views(self.v)
        step = 0
        with torch.no_grad():
            for i, st in d["state"].items():
                i = int(i)
                ms[i].copy_(st["exp_avg"])
                vs[i].copy_(st["exp_avg_sq"])
                step = int(float(st["step"]))
        self.step_dev.fill_(step)


class FusedPPOUpdate:
    """Drives the lgx PPO kernels for a standard rsl_rl ActorCritic (identical ELU hidden stacks
    for actor and critic)."""

    SPLITS = 8

    @staticmethod
    def supported(ac):
        def lin(seq):
            return [m for m in seq if isinstance(m, nn.Linear)], [m for m in seq if not isinstance(m, nn.Linear)]
        if getattr(ac, "is_recurrent", False) and (os.environ.get("LGX_PPO_FUSED_RECURRENT", "1") == "0"
                                                   or not hasattr(ac, "memory_a") or not hasattr(ac, "memory_c")):
            return False   # (LGX_PPO_FUSED_RECURRENT=0: recurrent policies on the autograd update)
        try:
            la, aa = lin(ac.actor)
            lc, acr = lin(ac.critic)
        except AttributeError:
            return False
        if not all(isinstance(m, nn.ELU) and m.alpha == 1.0 for m in aa + acr):
            return False
        if len(la) != len(lc) or len(la) < 2 or len(aa) != len(la) - 1 or len(acr) != len(lc) - 1:
            return False
        ha = [l.out_features for l in la[:-1]]
        hc = [l.out_features for l in lc[:-1]]
        L = len(ha)
        # one lgx_reduce_slices launch takes every gradient block: dW1 (x2 with a privileged critic
        # of another width), dW_2..L, the head dW, and the bias sums of every hidden layer; the
        # weight copies the Adam step maintains: padded W1 (x2) + transposed W_2..L
        sep = la[0].in_features != lc[0].in_features
        jobs = 2 * L + 1 + int(sep)
        mirrors = 2 * L - 1 + int(sep)     # split-bf16 limb copies: W_1 (x2), W_k and W_k^T
        return (ha == hc and all(h % 4 == 0 for h in ha) and ha[-1] <= 1024 and lc[-1].out_features == 1
                and la[-1].out_features <= abi.PPO_MAX_ACTIONS and ac.std.dim() == 1
                and jobs <= abi.MAX_REDUCE_JOBS and mirrors <= abi.MAX_REDUCE_JOBS)

    def __init__(self, ppo):
        from legged_gym_amd.sim import lib as lgxlib
        self.lib = lgxlib.load()
        self.check = lgxlib.check
        self.tuned = _TunedGemms()
        self.ppo = ppo
        ac = ppo.actor_critic
        self.dev = next(ac.parameters()).device
        la = [m for m in ac.actor if isinstance(m, nn.Linear)]
        lc = [m for m in ac.critic if isinstance(m, nn.Linear)]
        self.L = len(la) - 1                       # hidden layers
        self.hidden = [l.out_features for l in la[:-1]]
        self.num_obs = la[0].in_features
        self.num_cobs = lc[0].in_features
        self.A = la[-1].out_features
        # flat layout: layer-major so that {actor, critic} blocks of a layer are adjacent; the layer-1
        # biases right after the layer-1 weights: both come from dW1's lgx_gemm_tn (weights, and the
        # bias gradient from its column sums), so the second data-parallel gradient bucket - what
        # is complete only once dW1 is - is the contiguous prefix [0, nW1)
        order = [la[0].weight, lc[0].weight, la[0].bias, lc[0].bias]
        for k in range(1, self.L + 1):
            order += [la[k].weight, lc[k].weight]
        for k in range(1, self.L + 1):
            order += [la[k].bias, lc[k].bias]
        order.append(ac.std)
        # recurrent policies (ActorCriticRecurrent): the memories' parameters after the heads' (their
        # gradients come from torch autograd through the LSTM / GRU, fed with the heads' input
        # gradient dX = dZ_1 W_1 of the fused backward; the clip norm and Adam cover them too)
        self.recurrent = bool(getattr(ac, "is_recurrent", False))
        self.mem_params = (list(ac.memory_a.parameters()) + list(ac.memory_c.parameters())) if self.recurrent else []
        order += self.mem_params
        n = sum(p.numel() for p in order)
        self.flat_p = torch.zeros(n, device=self.dev)
        # gradient buffer + one trailing slot: the minibatch KL rides in the same all-reduce as the
        # gradient when data-parallel (one collective per minibatch)
        self.g_comm = torch.zeros(n + 1, device=self.dev)
        self.flat_g = self.g_comm[:n]
        self.off = {}
        off = 0
        with torch.no_grad():
            for p in order:
                k = p.numel()
                self.flat_p[off:off + k].copy_(p.data.reshape(-1))
                self.off[id(p)] = off
                p.data = self.flat_p[off:off + k].view_as(p)
                p.grad = self.flat_g[off:off + k].view_as(p)
                off += k
        self.n = n
        self.nW1 = self.off[id(la[1].weight)]   # end of the {actor, critic} layer-1 weight + bias blocks
        self.bucketed = False                     # (last minibatch: two all-reduce buckets)
        self.la, self.lc = la, lc
        self.W = []    # per layer k < L: stacked [2, out, in] weight view (k >= 1) or per-net views (k == 0)
        for k in range(self.L + 1):
            o = self.off[id(la[k].weight)]
            if k == 0 or k == self.L:
                self.W.append((la[k].weight, lc[k].weight))
            else:
                self.W.append(self.flat_p[o:o + 2 * la[k].weight.numel()].view(2, *la[k].weight.shape))
        self.Wg = [self.off[id(la[k].weight)] for k in range(self.L + 1)]
        if self.num_obs == self.num_cobs:
            o = self.Wg[0]
            self.W1s = self.flat_p[o:o + 2 * la[0].weight.numel()].view(2, *la[0].weight.shape)
        self.bo = [self.off[id(la[k].bias)] for k in range(self.L + 1)]
        self.std_off = self.off[id(ac.std)]
        params = list(ac.parameters())
        self.optimizer = FlatAdam(params, self.flat_p, self.flat_g, ppo.learning_rate)
        import os
        # LGX_PPO_GEMM: "lgx" (default) = every hidden-layer forward and backward dA on lgx_gemm_nt
        # (epilogues fused; measured ~1 % faster per iteration on MI355X than "auto"); "auto" =
        # lgx_gemm_nt for the layer-1 forward and the dA products, library GEMM + lgx_bias_act for
        # the other forwards; "lib" = none
        mode = os.environ.get("LGX_PPO_GEMM", "lgx")
        self.lgx_gemm = all(hk % abi.GEMM_TILE_N == 0 for hk in self.hidden) and mode != "lib"
        self.lgx_fwd_layers = set(range(self.L)) if mode == "lgx" else {0}
        # LGX_GEMM_ALGO: "split" (default) = lgx_gemm_nt's split-bf16 products (f32-accurate, bf16
        # MFMA) with pre-split weights; "f32" = the exact-f32 MFMA path with f32 weight copies
        self.split = os.environ.get("LGX_GEMM_ALGO", "split") != "f32"
        # LGX_PPO_DW: "lgx" (default with split-bf16 GEMMs) = weight gradients on lgx_gemm_tn
        # (split-bf16, transposed LDS reads); "lib" = library f32 bmm over row slices
        self.tn = self.lgx_gemm and self.split and os.environ.get("LGX_PPO_DW", "lgx") != "lib"
        self.gemm_dw = {}   # layer -> lgx_gemm_tn argument blocks (filled by _build_gemm_plan)
        self.norm_parts = torch.zeros(256, device=self.dev)
        self._mirrors_valid = False
        self.stats = torch.zeros(3, device=self.dev)
        self._pending = None      # a deferred update's readback (update(defer=True) -> resolve())
        self.M = None

    # ------------------------------------------------------------------ buffers
    def _alloc(self, M):
        if self.M == M:
            return
        dev, h, A = self.dev, self.hidden, self.A
        self.M = M
        # split-K row slices of each layer's dW GEMM (library bmm over slices, partials reduced in
        # lgx_reduce_slices): enough output tiles to fill the CUs. LGX_PPO_SPLITS="s1,s2,..." per layer
        env = os.environ.get("LGX_PPO_SPLITS")
        want = [int(x) for x in env.split(",")] if env else []
        self.Sk = []
        for k in range(self.L):
            # (dW on the side stream, next to the dA GEMMs: tiles for half the CUs - measured 10.32
            # -> 10.20 ms per update against a full CU round of tiles)
            fill = 0.5 if os.environ.get("LGX_PPO_DW_SIDE", "1") != "0" else 1.0
            sk = want[k] if k < len(want) else (self._tn_slices(h[k], h[k - 1] if k else self.num_obs, M, fill=fill)
                                                if self.tn else self.SPLITS)
            self.Sk.append(sk if sk > 0 and M % sk == 0 else 1)
        self.S = self.Sk[0]
        sep = self._separate_critic_obs()
        if self.lgx_gemm:   # K of layer 1 padded to the GEMM's K step with zero columns
            ks = abi.GEMM_K_STEP
            self.Kp, self.Kcp = -(-self.num_obs // ks) * ks, -(-self.num_cobs // ks) * ks
            self.Xp = torch.zeros(M, self.Kp, device=dev)
            self.X = self.Xp[:, :self.num_obs]
            self.Xcp = torch.zeros(M, self.Kcp, device=dev) if sep else None
            self.Xc = self.Xcp[:, :self.num_cobs] if sep else None
        else:
            self.X = torch.empty(M, self.num_obs, device=dev)
            self.Xc = torch.empty(M, self.num_cobs, device=dev) if sep else None
        self.Y = [torch.empty(2, M, hk, device=dev) for hk in h]
        self.D = [torch.empty(2, M, hk, device=dev) for hk in h[:-1]]
        self.MU = torch.empty(M, A, device=dev)
        self.V = torch.empty(M, 1, device=dev)
        self.dMU = torch.empty(M, A, device=dev)
        self.dV = torch.empty(M, device=dev)
        Sk = self.Sk
        # layer-1 dW partials: one [2, S, h0, K] block (one input for both networks), or (actor,
        # critic) blocks when the critic reads inputs of its own (privileged observations, of any
        # width; a recurrent policy's two memory outputs)
        p0 = (torch.empty(2, Sk[0], h[0], self.num_obs, device=dev) if self.num_cobs == self.num_obs and not sep else
              (torch.empty(Sk[0], h[0], self.num_obs, device=dev), torch.empty(Sk[0], h[0], self.num_cobs, device=dev)))
        self.P = [p0] + \
                 [torch.empty(2 * Sk[k], h[k], h[k - 1], device=dev) for k in range(1, self.L)]
        # output layers evaluated inside the loss call (no head GEMM launches) when they fit its LDS;
        # with them, loss + output-layer backward in one launch (lgx_ppo_loss_bwd, its loss finalize
        # in the reduction launch) unless LGX_PPO_LOSS_BWD=0
        H = h[-1]
        self.head_in_loss = (os.environ.get("LGX_PPO_HEAD_IN_LOSS", "1") != "0" and H % 16 == 0
                             and (A + 1) * H * 4 <= 65536)
        lay = (C.c_int64 * 3)()
        self.check(self.lib.lgx_ppo_loss_bwd_layout(M, A, H, lay), "loss_bwd_layout")
        self.loss_bwd = self.head_in_loss and lay[2] <= 96 * 1024 and os.environ.get("LGX_PPO_LOSS_BWD", "1") != "0"
        if self.loss_bwd:
            self.loss_parts = torch.empty(int(lay[0]), device=dev)
            self.head_parts = torch.empty(int(lay[1]), device=dev)
        else:
            self.loss_parts = torch.empty(int(self.lib.lgx_ppo_loss_partials_floats(M, A)), device=dev)
            self.head_parts = torch.empty(int(self.lib.lgx_head_bwd_partials_floats(M, A, H)), device=dev)
        if self.lgx_gemm:
            self.col_parts = [torch.empty(int(self.lib.lgx_gemm_partials_floats(M, hk, 2)), device=dev)
                              for hk in h[:-1]]
            self._build_gemm_plan()
        else:
            self.col_parts = [torch.empty(int(self.lib.lgx_colsum_partials_floats(M, hk, 2)), device=dev)
                              for hk in h[:-1]]
        self._build_reduce_jobs()

    @staticmethod
    def _tn_slices(R, Cc, M, cus=256, fill=1.0):
        """Row slices of one lgx_gemm_tn launch: the fewest (>= 8, powers of 2) that give a
        fraction `fill` of the CUs an output tile (R/128 x ceil(Cc/128) tiles per slice and
        network) with 32-row multiples."""
        tiles = (R // (256 if R % 256 == 0 else 128)) * (-(-Cc // 128)) * 2   # lgx_gemm_tn tile rows
        s = 8
        while tiles * s < cus * fill and M % (2 * s * 32) == 0:
            s *= 2
        while s > 1 and M % (s * 32):   # small minibatches: fewer slices of 32-row multiples
            s //= 2
        return s

    def _build_gemm_plan(self):
        """Fixed argument blocks of every lgx_gemm_nt / lgx_copy2d launch of a minibatch (the
        buffers do not move, so a minibatch issues the prepared structs)."""
        M, h, L, dev = self.M, self.hidden, self.L, self.dev
        fp = self.flat_p
        f4 = 4
        shared = self.Xcp is None and self.num_obs == self.num_cobs
        copies = []

        def copy(src_ptr, dst, rows, cols, batch, transpose, src_ld, dst_ld):
            j = abi.LgxCopy2dJob()
            j.src, j.dst = src_ptr, dst.data_ptr()
            j.src_ld, j.src_bs = src_ld, rows * cols
            j.dst_ld, j.dst_bs = dst_ld, (cols if transpose else rows) * dst_ld
            j.rows, j.cols, j.batch, j.transpose = rows, cols, batch, int(transpose)
            copies.append(j)
        w1 = fp.data_ptr() + f4 * self.Wg[0]
        nl = [None] * (L + 1)   # split-bf16: limb copies of W_1 / W_k (forward) and W_k^T (backward dA)
        nlt = [None] * (L + 1)
        if self.split:
            # the B operands pre-split into bf16 limbs (lgx_split_bf16 before an update's first
            # minibatch, then kept current by the Adam step's limb mirrors: transpose bit 1)
            def limbs(src_ptr, rows, cols, batch, transpose):
                nout, kout = (cols, rows) if transpose else (rows, cols)
                ld = int(self.lib.lgx_split_bf16_elems(1, kout))
                buf = torch.zeros(batch * nout * ld, dtype=torch.int16, device=dev)
                j = abi.LgxCopy2dJob()
                j.src, j.dst = src_ptr, buf.data_ptr()
                j.src_ld, j.src_bs, j.dst_ld, j.dst_bs = cols, rows * cols, ld, nout * ld
                j.rows, j.cols, j.batch, j.transpose = rows, cols, batch, int(transpose) | 2
                copies.append(j)
                return buf
            if shared:
                nl[0] = (limbs(w1, h[0], self.num_obs, 2, False),)
            else:
                nl[0] = (limbs(w1, h[0], self.num_obs, 1, False),
                         limbs(w1 + f4 * h[0] * self.num_obs, h[0], self.num_cobs, 1, False))
            for k in range(1, L):
                wk = fp.data_ptr() + f4 * self.Wg[k]
                nl[k] = limbs(wk, h[k], h[k - 1], 2, False)
                nlt[k] = limbs(wk, h[k], h[k - 1], 2, True)
            self.limb_bufs = (nl, nlt)
        else:
            if shared:
                self.W1p = torch.zeros(2, h[0], self.Kp, device=dev)
                copy(w1, self.W1p, h[0], self.num_obs, 2, False, self.num_obs, self.Kp)
            else:
                self.W1p = torch.zeros(h[0], self.Kp, device=dev)
                self.W1pc = torch.zeros(h[0], self.Kcp, device=dev)
                copy(w1, self.W1p, h[0], self.num_obs, 1, False, self.num_obs, self.Kp)
                copy(w1 + f4 * h[0] * self.num_obs, self.W1pc, h[0], self.num_cobs, 1, False, self.num_cobs, self.Kcp)
            self.WT = [None]
            for k in range(1, L):   # W_k [2, h_k, h_{k-1}] -> W_k^T [2, h_{k-1}, h_k]
                wt = torch.empty(2, h[k - 1], h[k], device=dev)
                copy(fp.data_ptr() + f4 * self.Wg[k], wt, h[k], h[k - 1], 2, True, h[k - 1], h[k])
                self.WT.append(wt)
        if len(copies) > abi.MAX_REDUCE_JOBS:
            raise RuntimeError("too many weight-preparation jobs for one launch")
        self.copy_jobs = (abi.LgxCopy2dJob * len(copies))(*copies)
        algo = abi.GEMM_ALGO_SPLIT_BF16 if self.split else abi.GEMM_ALGO_F32

        def gemm(A, lda, sa, B, ldb, sb, C, N, K, batch, epi, bias=None, Y=None, parts=None, Bs=None):
            g = abi.LgxGemmArgs()
            g.M, g.N, g.K, g.batch, g.epi = M, N, K, batch, epi
            g.A, g.lda, g.sa = A, lda, sa
            g.B, g.ldb, g.sb = B, ldb, sb
            g.C, g.ldc, g.sc = C.data_ptr(), N, M * N
            g.bias = bias
            g.Y = Y.data_ptr() if Y is not None else None
            g.partials = parts.data_ptr() if parts is not None else None
            g.algo = algo
            g.Bs = Bs.data_ptr() if Bs is not None else None
            return g
        fwd = [[]]
        b0 = fp.data_ptr() + f4 * self.bo[0]
        self.fwd0_src = ["x"] if shared else ["x", "xc"]
        w1p = None if self.split else self.W1p.data_ptr()
        if shared:   # one input for both networks: batch stride 0
            fwd[0].append(gemm(self.Xp.data_ptr(), self.Kp, 0, w1p, self.Kp, h[0] * self.Kp, self.Y[0],
                               h[0], self.Kp, 2, abi.GEMM_BIAS_ELU, bias=b0, Bs=nl[0][0] if self.split else None))
        else:
            fwd[0].append(gemm(self.Xp.data_ptr(), self.Kp, 0, w1p, self.Kp, 0, self.Y[0][0], h[0],
                               self.Kp, 1, abi.GEMM_BIAS_ELU, bias=b0, Bs=nl[0][0] if self.split else None))
            xc = self.Xcp if self.Xcp is not None else self.Xp
            fwd[0].append(gemm(xc.data_ptr(), self.Kcp, 0, None if self.split else self.W1pc.data_ptr(), self.Kcp, 0,
                               self.Y[0][1], h[0], self.Kcp, 1, abi.GEMM_BIAS_ELU, bias=b0 + f4 * h[0],
                               Bs=nl[0][1] if self.split else None))
        for k in range(1, L):
            fwd.append(gemm(self.Y[k - 1].data_ptr(), h[k - 1], M * h[k - 1], fp.data_ptr() + f4 * self.Wg[k], h[k - 1],
                            h[k] * h[k - 1], self.Y[k], h[k], h[k - 1], 2, abi.GEMM_BIAS_ELU,
                            bias=fp.data_ptr() + f4 * self.bo[k], Bs=nl[k]))
        self.gemm_fwd = fwd
        # algorithmic K of each launch (layer 1: the unpadded input width) for the bench's roofline
        self.k_alg = {id(g): k for g, k in zip(fwd[0], [self.num_obs, self.num_cobs])}
        # weight gradients (lgx_gemm_tn): dW_k = dZ_k^T Y_{k-1} over Sk row slices into P[k]
        self.gemm_dw = {}
        if self.tn:
            def tn(A, lda, sa, B, ldb, sb, Cp, R, Cc, S, batch):
                t = abi.LgxGemmTnArgs()
                t.M, t.R, t.Cc, t.slices, t.batch = M, R, Cc, S, batch
                t.A, t.lda, t.sa = A, lda, sa
                t.B, t.ldb, t.sb = B, ldb, sb
                t.C, t.ldc = Cp, Cc
                return t
            tn_ok = [M % (self.Sk[k] * 32) == 0 for k in range(L)]   # else the library bmm (rows % 32)
            for k in range(L - 1, 0, -1):
                if not tn_ok[k]:
                    continue
                dz = self.Y[L - 1] if k == L - 1 else self.D[k]
                self.gemm_dw[k] = [tn(dz.data_ptr(), h[k], M * h[k], self.Y[k - 1].data_ptr(), h[k - 1], M * h[k - 1],
                                      self.P[k].data_ptr(), h[k], h[k - 1], self.Sk[k], 2)]
            # layer 1: B = the minibatch's padded input rows (pointer set per minibatch); the padding
            # columns up to the next multiple of 128 must exist in the rows
            if tn_ok[0] and self.Kp >= -(-self.num_obs // 128) * 128 and (
                    self.Xcp is None or self.Kcp >= -(-self.num_cobs // 128) * 128):
                d0 = self.D[0]
                if isinstance(self.P[0], tuple):     # privileged critic inputs: one launch per network
                    self.gemm_dw[0] = [tn(d0[0].data_ptr(), h[0], 0, 0, self.Kp, 0, self.P[0][0].data_ptr(), h[0],
                                          self.num_obs, self.Sk[0], 1),
                                       tn(d0[1].data_ptr(), h[0], 0, 0, self.Kcp, 0, self.P[0][1].data_ptr(), h[0],
                                          self.num_cobs, self.Sk[0], 1)]
                else:                                # one input for both networks: batch stride 0
                    self.gemm_dw[0] = [tn(d0.data_ptr(), h[0], M * h[0], 0, self.Kp, 0, self.P[0].data_ptr(), h[0],
                                          self.num_obs, self.Sk[0], 2)]
        # bias gradients db_k of the hidden layers below the last: the column sums of dZ_k, taken by
        # dW_k's lgx_gemm_tn from the rows it stages anyway (per-slice partials, reduced with the
        # weight gradients); the dA GEMM producing dZ_k then runs the plain ELU' epilogue
        # (LGX_GEMM_DELU: transposed accumulators, output deferred into the next tile's slots).
        # Layers whose dW is not on lgx_gemm_tn keep the ELU' + column-sum epilogue.
        self.colsum = {}
        if self.split and os.environ.get("LGX_PPO_TN_COLSUM", "1") != "0":
            for k in range(L - 1):
                if k not in self.gemm_dw:
                    continue
                cs = torch.empty(2, self.Sk[k], h[k], device=dev)
                self.colsum[k] = cs
                for z, t in enumerate(self.gemm_dw[k]):   # (batch 2, or one launch per network)
                    t.colsum = cs.data_ptr() + 4 * z * self.Sk[k] * h[k]
        bwd = {}
        for k in range(L - 1, 0, -1):   # dZ_{k-1} = (dZ_k W_k) * elu'(Y_{k-1}); dZ_{L-1} lives in Y[L-1]
            dz = self.Y[L - 1] if k == L - 1 else self.D[k]
            plain = (k - 1) in self.colsum
            bwd[k] = gemm(dz.data_ptr(), h[k], M * h[k], None if self.split else self.WT[k].data_ptr(), h[k],
                          h[k - 1] * h[k], self.D[k - 1], h[k - 1], h[k], 2,
                          abi.GEMM_DELU if plain else abi.GEMM_DELU_COLSUM, Y=self.Y[k - 1],
                          parts=None if plain else self.col_parts[k - 1], Bs=nlt[k])
        self.gemm_bwd = bwd

    def _separate_critic_obs(self):
        if self.recurrent:   # the heads' inputs are the two memories' outputs
            return True
        st = self.ppo.storage
        return st is not None and st.privileged_observations is not None

    def _build_reduce_jobs(self):
        M, S, h, A = self.M, self.S, self.hidden, self.A
        g = self.flat_g
        jobs = []

        def job(src, dst_off, n, count, job_stride, slices, slice_stride, dst_stride):
            j = abi.LgxReduceJob()
            j.src = src.data_ptr()
            j.dst = g.data_ptr() + 4 * dst_off
            j.n, j.count, j.job_stride, j.slices, j.slice_stride, j.dst_stride = n, count, job_stride, slices, \
                slice_stride, dst_stride
            jobs.append(j)
        n1 = h[0] * self.num_obs
        Sk = self.Sk
        if isinstance(self.P[0], tuple):                                             # dW1 actor, critic
            n1c = h[0] * self.num_cobs
            job(self.P[0][0], self.Wg[0], n1, 1, 0, Sk[0], n1, 0)
            job(self.P[0][1], self.Wg[0] + n1, n1c, 1, 0, Sk[0], n1c, 0)
        else:
            job(self.P[0], self.Wg[0], n1, 2, Sk[0] * n1, Sk[0], n1, n1)            # dW1 (actor, critic)
        colsum = getattr(self, "colsum", {})
        if 0 in colsum:   # db_1 from dW1's column sums: complete with dW1
            job(colsum[0], self.bo[0], h[0], 2, Sk[0] * h[0], Sk[0], h[0], h[0])
        elif self.L > 1:
            # db_1 from the dA_1 GEMM's ELU' + column-sum partials (dW1 not on lgx_gemm_tn: e.g. 48 or
            # 169 observations, whose padded rows are narrower than dW1's 128-column tiles).  dA_1 runs
            # on the main stream after the side stream's last join, so this job belongs with dW1's on
            # the main stream: reduced after dA_1, and inside the [0, nW1) all-reduce bucket that is
            # issued from the main stream (in the side stream's early reduction it would read the
            # partials before dA_1 wrote them)
            cchunks = self.col_parts[0].numel() // (2 * h[0])
            job(self.col_parts[0], self.bo[0], 2 * h[0], 1, 0, cchunks, 2 * h[0], 0)
        n_dw1 = len(jobs)   # (the layer-1 jobs come first: the rest can be reduced before dW1 is done)
        for k in range(1, self.L):
            nk = h[k] * h[k - 1]
            job(self.P[k], self.Wg[k], nk, 2, Sk[k] * nk, Sk[k], nk, nk)            # dW_k stacked
        nh = (A + 1) * h[-1] + 2 * h[-1]
        hchunks = self.head_parts.numel() // nh                                     # per-chunk partial rows
        job(self.head_parts, self.Wg[self.L], (A + 1) * h[-1], 1, 0, hchunks, nh, 0)  # dW head (actor | critic)
        hp_b = self.head_parts[(A + 1) * h[-1]:]
        job(hp_b, self.bo[self.L - 1], 2 * h[-1], 1, 0, hchunks, nh, 0)              # db of the last hidden layer
        for k in range(1, self.L - 1):   # (db_1 is with the layer-1 jobs above)
            if k in colsum:                                                          # db_k from dW_k's column sums
                job(colsum[k], self.bo[k], h[k], 2, Sk[k] * h[k], Sk[k], h[k], h[k])
                continue
            cchunks = self.col_parts[k].numel() // (2 * h[k])
            job(self.col_parts[k], self.bo[k], 2 * h[k], 1, 0, cchunks, 2 * h[k], 0)  # db_k
        if len(jobs) > abi.MAX_REDUCE_JOBS:
            raise RuntimeError("too many reduction jobs for one launch")
        self.jobs = (abi.LgxReduceJob * len(jobs))(*jobs)
        self.njobs = len(jobs)
        self.jobs_dw1 = (abi.LgxReduceJob * n_dw1)(*jobs[:n_dw1])
        self.jobs_rest = (abi.LgxReduceJob * (len(jobs) - n_dw1))(*jobs[n_dw1:])
        # every input of jobs_rest comes from the side stream's dW launches (partials, column sums)
        # or from launches on the main stream before the side stream's first join (loss): the
        # early reduction then needs no join after the dA GEMMs.  (db_k from a dA epilogue, k >= 2,
        # is written on the main stream after a join: then the join is needed; db_1 is never in
        # jobs_rest.)
        self.rest_on_side = all(k in colsum for k in range(1, self.L - 1))
        # the clip norm's sums of squares written by the reduction launches themselves
        # (lgx_reduce_slices_sq; single-process updates with the fused loss): one launch less per minibatch
        self.fused_sq = (self.lgx_gemm and self.loss_bwd and not self.recurrent
                         and os.environ.get("LGX_PPO_FUSED_SQ", "1") != "0")
        if self.fused_sq:
            blocks = self.lib.lgx_reduce_slices_blocks
            self.nsq_rest = int(blocks(self.jobs_rest, len(self.jobs_rest), 1)) if len(self.jobs_rest) else 0
            self.nsq_dw1 = int(blocks(self.jobs_dw1, len(self.jobs_dw1), 0))
            self.nsq_all = int(blocks(self.jobs, self.njobs, 1))
            if min(self.nsq_rest, self.nsq_dw1, self.nsq_all) < 0:
                raise RuntimeError("lgx_reduce_slices_blocks failed")
            self.sq_parts = torch.zeros(max(self.nsq_rest + self.nsq_dw1, self.nsq_all, 1), device=self.dev)

    # ------------------------------------------------------------------ update
    @torch.no_grad()
    def update(self, defer=False):
        """One PPO update (rsl_rl PPO.update).  Returns (mean value loss, mean surrogate loss) after
        reading the statistics and the adapted learning rate back (one host synchronisation).
        defer=True returns None right after issuing: the readback goes to pinned host memory behind
        an event and resolve() - called by the next update() or by the caller - applies it, so the
        host can issue the next rollout while this update still runs (the GPU otherwise idles at the
        iteration boundary until the host returns from the synchronisation and issues again)."""
        self.resolve()   # (a previous deferred update finished long before this one is issued)
        if self.recurrent:
            return self._update_recurrent(defer)
        t_issue = time.perf_counter()
        ppo = self.ppo
        st = ppo.storage
        T, N = st.num_transitions_per_env, st.num_envs
        B = T * N
        nmb = ppo.num_mini_batches
        M = B // nmb
        self._alloc(M)
        self._mirrors_valid = False      # parameters may have changed since the last update
        stream = C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        if ppo.desired_kl is not None and ppo.schedule == "adaptive":
            self.optimizer.lr_dev.fill_(ppo.learning_rate)
        # (fixed schedule: lr_dev keeps the optimizer's lr, i.e. a checkpoint's after load_state_dict,
        # as torch.optim.Adam's param_groups do)
        self.stats.zero_()
        # as rsl_rl's generator; drawn on a second stream (the generator's offset is taken at issue,
        # so the permutation is the same on any stream): its sort chain of small launches runs next
        # to the rollout's last steps / GAE still queued on this stream instead of after them
        main = torch.cuda.current_stream(self.dev)
        if getattr(self, "_perm_stream", None) is None:
            self._perm_stream = torch.cuda.Stream(self.dev)
        with torch.cuda.stream(self._perm_stream):
            indices = torch.randperm(nmb * M, requires_grad=False, device=self.dev)
        main.wait_stream(self._perm_stream)
        indices.record_stream(main)
        obs = st.observations.view(B, -1)
        cobs = st.privileged_observations.view(B, -1) if st.privileged_observations is not None else None
        storage = dict(actions=st.actions.view(B, -1), old_logp=st.actions_log_prob.view(B),
                       old_mu=st.mu.view(B, -1), old_sigma=st.sigma.view(B, -1), advantages=st.advantages.view(B),
                       target_values=st.values.view(B), returns=st.returns.view(B))
        args = self._loss_args(storage)
        xs = None
        if self.lgx_gemm:
            # rsl_rl draws ONE permutation per update and every epoch walks the same minibatches,
            # so the padded layer-1 inputs are gathered once (one launch over all B rows) and a
            # minibatch reads its contiguous slice: no per-minibatch gather
            xs = self._gather_all(indices, obs, cobs, nmb * M, stream)
        for _ in range(ppo.num_learning_epochs):
            for i in range(nmb):
                idx = indices[i * M:(i + 1) * M]
                if xs is None:
                    mx = None
                elif self.dw1_batched:        # [2, M, Kp] block: the same rows for actor and critic
                    mx = (xs[0][i], None, xs[0][i])
                else:
                    mx = tuple(x[i * M:(i + 1) * M] if x is not None else None for x in xs)
                self._minibatch(idx, obs, cobs, args, stream, xs=mx)
        self.host_issue_s = time.perf_counter() - t_issue   # host time to issue every launch (tools/host_overhead.py)
        return self._finish(ppo.num_learning_epochs * nmb, defer)

    def _finish(self, n, defer):
        """The update's readback (statistics, adapted learning rate) over its n minibatches: now, or
        deferred to pinned memory behind an event (resolve())."""
        if not defer:
            return self._apply_readback(self.stats.tolist(), float(self.optimizer.lr_dev.item()), n)
        if getattr(self, "_pin_stats", None) is None:
            self._pin_stats = torch.empty(self.stats.shape, dtype=self.stats.dtype).pin_memory()
            self._pin_lr = torch.empty(1, dtype=self.optimizer.lr_dev.dtype).pin_memory()
            self._pin_ev = torch.cuda.Event()
        self._pin_stats.copy_(self.stats, non_blocking=True)
        self._pin_lr.copy_(self.optimizer.lr_dev.view(1), non_blocking=True)
        self._pin_ev.record(torch.cuda.current_stream(self.dev))
        self._pending = n
        return None


    # ------------------------------------------------------------------ recurrent policies
    def _rec_rows(self, i, T, N, envs):
        """Storage rows of recurrent minibatch i in the heads' row order (t-major over the envs
        [i envs, (i + 1) envs): the unpadded memory output [T, envs, H] flattened)."""
        cache = getattr(self, "_rec_idx", None)
        if cache is None or cache[0] != (T, N, envs):
            cache = ((T, N, envs), {})
            self._rec_idx = cache
        if i not in cache[1]:
            t = torch.arange(T, device=self.dev, dtype=torch.int64)[:, None] * N
            cache[1][i] = (t + i * envs + torch.arange(envs, device=self.dev, dtype=torch.int64)[None, :]).reshape(-1)
        return cache[1][i]

    def _update_recurrent(self, defer):
        """rsl_rl PPO.update for ActorCriticRecurrent (reccurent_mini_batch_generator: minibatches of
        whole envs in order, padded trajectories, the memories' saved first-step states).  Per
        minibatch the LSTM / GRU runs forward on torch with autograd (the heads' inputs), the heads
        run the fused forward / loss / backward of a feed-forward policy on those inputs, and
        _memory_backward carries dX = dZ_1 W_1 back through the memories into the flat gradient
        before the clip norm and Adam."""
        t_issue = time.perf_counter()
        ppo, ac = self.ppo, self.ppo.actor_critic
        st = ppo.storage
        T, N = st.num_transitions_per_env, st.num_envs
        B = T * N
        nmb = ppo.num_mini_batches
        envs = N // nmb
        M = T * envs
        self._alloc(M)
        self._mirrors_valid = False
        stream = C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        if ppo.desired_kl is not None and ppo.schedule == "adaptive":
            self.optimizer.lr_dev.fill_(ppo.learning_rate)
        self.stats.zero_()
        storage = dict(actions=st.actions.view(B, -1), old_logp=st.actions_log_prob.view(B),
                       old_mu=st.mu.view(B, -1), old_sigma=st.sigma.view(B, -1), advantages=st.advantages.view(B),
                       target_values=st.values.view(B), returns=st.returns.view(B))
        args = self._loss_args(storage)
        H = self.num_obs
        k = 0
        for (obs_b, cobs_b, _a, _v, _adv, _r, _lp, _mu, _sg, hid_b, masks_b) in \
                st.reccurent_mini_batch_generator(nmb, ppo.num_learning_epochs):
            i = k % nmb
            k += 1
            with torch.enable_grad():
                xa = ac.memory_a(obs_b, masks_b, hid_b[0])       # [T, envs, H]
                xc = ac.memory_c(cobs_b, masks_b, hid_b[1])
            xs = []
            for x, pad in ((xa, self.Xp), (xc, self.Xcp)):
                x2 = x.detach().reshape(M, H)
                if pad.shape[1] == H and x2.is_contiguous() and x2.data_ptr() % 16 == 0:
                    xs.append(x2)
                else:                              # (K padded to the GEMM step: zero columns stay)
                    pad[:, :H].copy_(x2)
                    xs.append(pad)
            self._mem_ctx = (xa, xc)
            self._mem_xs = xs      # (the heads' input rows stay referenced until the next minibatch)
            self._minibatch(self._rec_rows(i, T, N, envs), None, None, args, stream, xs=(xs[0], xs[1]))
            self._mem_ctx = None
        self.host_issue_s = time.perf_counter() - t_issue
        return self._finish(ppo.num_learning_epochs * nmb, defer)

    def _memory_backward(self):
        """The memories' gradients of a recurrent minibatch: dX = dZ_1 W_1 per network (the heads'
        input gradient; dZ_1 from the fused backward), then torch autograd through the LSTM / GRU
        forward of this minibatch, written into the memories' blocks of the flat gradient (every
        other block is complete: this runs after the reductions, on the update's stream)."""
        ctx = getattr(self, "_mem_ctx", None)
        if ctx is None:
            return
        xa, xc = ctx
        dz1 = self.D[0] if self.L > 1 else self.Y[self.L - 1]        # [2, M, h1]
        wa, wc = self.W[0]                                           # [h1, H] each
        dxa = torch.mm(dz1[0], wa).view_as(xa)
        dxc = torch.mm(dz1[1], wc).view_as(xc)
        with torch.enable_grad():
            grads = torch.autograd.grad([xa, xc], self.mem_params, grad_outputs=[dxa, dxc], allow_unused=True)
        for p, g in zip(self.mem_params, grads):
            if g is None:
                p.grad.zero_()
            else:
                p.grad.copy_(g)

    def _apply_readback(self, s, lr, n):
        ppo = self.ppo
        if ppo.desired_kl is not None and ppo.schedule == "adaptive":
            ppo.learning_rate = lr
        self.optimizer.param_groups[0]["lr"] = lr
        self.last_losses = (s[2] / n, s[1] / n)
        return self.last_losses

    def resolve(self):
        """Apply a deferred update's readback (learning rate, losses); returns its losses, or None
        when nothing is pending."""
        n, self._pending = self._pending, None
        if n is None:
            return None
        self._pin_ev.synchronize()
        return self._apply_readback(self._pin_stats.tolist(), float(self._pin_lr[0]), n)

    def _gather_all(self, indices, obs, cobs, rows, stream):
        # one input for both networks: rows gathered twice per minibatch ([nmb, 2, M, Kp]) so the
        # layer-1 weight gradients of actor and critic are ONE batched split-K GEMM
        self.dw1_batched = (cobs is None and self.num_obs == self.num_cobs and self.Xcp is None and 0 not in self.gemm_dw
                            and os.environ.get("LGX_PPO_DW1_BATCHED", "1") != "0")
        if self.dw1_batched:
            M = self.M
            if getattr(self, "Xall2", None) is None or self.Xall2.shape[0] * M != rows:
                self.Xall2 = torch.zeros(rows // M, 2, M, self.Kp, device=self.dev)
            self.check(self.lib.lgx_ppo_gather_rows_padded_dup(_vp(obs), _vp(self.Xall2), _vp(indices), rows,
                                                               obs.shape[1], self.Kp, M, stream), "gather")
            return self.Xall2, None
        if getattr(self, "Xall", None) is None or self.Xall.shape[0] != rows:
            self.Xall = torch.zeros(rows, self.Kp, device=self.dev)     # padding columns stay zero
            self.Xcall = torch.zeros(rows, self.Kcp, device=self.dev) if self.Xcp is not None else None
        self.check(self.lib.lgx_ppo_gather_rows_padded(_vp(obs), _vp(self.Xall), _vp(indices), rows, obs.shape[1],
                                                       self.Kp, stream), "gather")
        if cobs is not None:
            self.check(self.lib.lgx_ppo_gather_rows_padded(_vp(cobs), _vp(self.Xcall), _vp(indices), rows,
                                                           cobs.shape[1], self.Kcp, stream), "gather")
        return self.Xall, self.Xcall

    def _loss_args(self, storage):
        a = abi.LgxPpoLossArgs()
        p = self.ppo
        a.rows, a.num_actions = self.M, self.A
        a.use_clipped_value_loss = int(bool(p.use_clipped_value_loss))
        a.clip_param, a.value_loss_coef, a.entropy_coef = p.clip_param, p.value_loss_coef, p.entropy_coef
        a.mu_raw, a.v_raw = self.MU.data_ptr(), self.V.data_ptr()
        a.b4a = self.flat_p.data_ptr() + 4 * self.bo[self.L]
        a.b4c = a.b4a + 4 * self.A
        a.std = self.flat_p.data_ptr() + 4 * self.std_off
        for k, v in storage.items():
            setattr(a, k, v.data_ptr())
        a.d_mu, a.d_v, a.partials = self.dMU.data_ptr(), self.dV.data_ptr(), self.loss_parts.data_ptr()
        a.g_b4a = self.flat_g.data_ptr() + 4 * self.bo[self.L]
        a.g_b4c = a.g_b4a + 4 * self.A
        a.g_std = self.flat_g.data_ptr() + 4 * self.std_off
        a.stats = self.stats.data_ptr()
        H = self.hidden[-1]
        if self.head_in_loss:   # (decided in _alloc)
            a.head_in, a.hidden = self.Y[self.L - 1].data_ptr(), H
            a.W4a, a.W4c = self.W[self.L][0].data_ptr(), self.W[self.L][1].data_ptr()
        else:
            a.head_in, a.W4a, a.W4c, a.hidden = None, None, None, 0
        a.defer_finalize = 1     # run by lgx_head_bwd_finalize / lgx_reduce_slices_finalize
        # single process with the adaptive schedule: the loss finalize adapts the learning rate
        # (data-parallel: lgx_ppo_adapt_lr after the all-reduce the KL rides in)
        if p.desired_kl is not None and p.schedule == "adaptive" and p.dist is None:
            a.lr, a.desired_kl = self.optimizer.lr_dev.data_ptr(), float(p.desired_kl)
        else:
            a.lr, a.desired_kl = None, 0.0
        self._keep = storage
        return a

    def gradients(self, idx, apply=False):
        """Flat gradient of one minibatch (rows `idx` of the current storage), for tests."""
        if self.recurrent:   # (a recurrent minibatch is whole envs through the memories: update())
            raise NotImplementedError("gradients(idx) takes feed-forward policies; recurrent ones go through update()")
        st = self.ppo.storage
        T, N = st.num_transitions_per_env, st.num_envs
        B = T * N
        self._alloc(idx.numel())
        self._mirrors_valid = False
        stream = C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        obs = st.observations.view(B, -1)
        cobs = st.privileged_observations.view(B, -1) if st.privileged_observations is not None else None
        storage = dict(actions=st.actions.view(B, -1), old_logp=st.actions_log_prob.view(B),
                       old_mu=st.mu.view(B, -1), old_sigma=st.sigma.view(B, -1), advantages=st.advantages.view(B),
                       target_values=st.values.view(B), returns=st.returns.view(B))
        self._minibatch(idx, obs, cobs, self._loss_args(storage), stream, apply=apply)
        return self.flat_g.clone()

    # ------------------------------------------------------------------ GEMM timing (bench.py)
    def time_gemms(self, period):
        """Bracket every lgx_gemm_nt launch of every `period`-th minibatch with HIP events on the
        launch stream (0: off); gemm_timings() reads them back per epilogue (kernel instantiation).
        The data-parallel gradient all-reduces of those minibatches are bracketed too
        (comm_timings())."""
        self._t_period, self._t_count, self._t_events, self._t_mb = int(period), 0, [], 0
        self._c_events = []

    def _all_reduce(self, buf, torch_stream):
        """ppo.dist.all_reduce(buf) issued on `torch_stream` (the current stream), with HIP events
        around it on that stream when this minibatch is timed."""
        rec = getattr(self, "_t_period", 0) and self._t_count % self._t_period == 0
        if rec:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch_stream)
        comm = self._lgx_comm()
        if comm is not None:   # lgx_allreduce_grads: RCCL on this stream itself (sum; 1/world in Adam)
            assert buf.dtype == torch.float32 and buf.is_contiguous()
            # one communicator, collectives issued from two streams (the bucketed update: side, then
            # main): RCCL orders nothing across streams, so a collective issued from another stream
            # than the previous one waits for it (torch's process group serialises on its own stream)
            prev = getattr(self, "_comm_last", None)
            if prev is not None and prev[0] != torch_stream.cuda_stream:
                torch_stream.wait_event(prev[1])
            self.check(self.lib.lgx_allreduce_grads(comm, _vp(buf), buf.numel(), 0,
                                                    C.c_void_p(torch_stream.cuda_stream)), "allreduce_grads")
            done = torch.cuda.Event()
            done.record(torch_stream)
            self._comm_last = (torch_stream.cuda_stream, done)
        else:
            self.ppo.dist.all_reduce(buf)
        if rec:
            e1.record(torch_stream)
            self._c_events.append((buf.numel() * buf.element_size(), e0, e1))

    @property
    def allreduce_impl(self):
        """"lgx" (lgx_allreduce_grads on the library's own RCCL communicator, LGX_NATIVE_ALLREDUCE=1
        with the nccl backend) or "torch" (torch.distributed.all_reduce, the default)."""
        return "lgx" if getattr(self, "_comm", None) is not None else "torch"

    def _lgx_comm(self):
        """The rank's lgx_comm, created collectively at the first gradient all-reduce when
        LGX_NATIVE_ALLREDUCE=1 and the process group is nccl (RCCL): rank 0 draws the unique id,
        the group broadcasts it; the RCCL library is torch's own (one RCCL instance per process)."""
        if hasattr(self, "_comm"):
            return self._comm
        self._comm = None
        dist = self.ppo.dist
        if os.environ.get("LGX_NATIVE_ALLREDUCE", "0") != "1":
            return None
        # asked for: fail loudly rather than fall back to torch.distributed (the 8-GPU run must use
        # the path it was configured for) or load an RCCL other than the one torch's nccl backend runs
        if dist.get_backend() != "nccl":
            raise RuntimeError(f"LGX_NATIVE_ALLREDUCE=1 needs the nccl (RCCL) process group, got {dist.get_backend()!r}")
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            raise RuntimeError(f"LGX_NATIVE_ALLREDUCE=1: torch's RCCL ({path}) is missing; refusing to load another "
                               "RCCL instance into the process")
        path = path.encode()
        uid = torch.zeros(128, dtype=torch.uint8)
        if dist.get_rank() == 0:
            self.check(self.lib.lgx_comm_unique_id(path, C.cast(uid.data_ptr(), C.POINTER(C.c_uint8))),
                       "comm_unique_id")
        dev_uid = uid.to(self.dev)
        dist.broadcast(dev_uid, src=0)
        uid = dev_uid.cpu()
        comm = C.c_void_p()
        self.check(self.lib.lgx_comm_create(path, C.cast(uid.data_ptr(), C.POINTER(C.c_uint8)), dist.get_world_size(),
                                            dist.get_rank(), self.dev.index or 0, C.byref(comm)), "comm_create")
        self._comm = comm
        return comm

    def close_comm(self):
        """Destroy the lgx_comm (collective: every rank calls it after its last update)."""
        comm, self._comm = getattr(self, "_comm", None), None
        if comm is not None:
            torch.cuda.synchronize(self.dev)
            self.check(self.lib.lgx_comm_destroy(comm), "comm_destroy")

    def comm_timings(self):
        """(collectives timed, total ms, total bytes, timed minibatches) of the all-reduces of the
        timed minibatches."""
        torch.cuda.synchronize()
        ev = getattr(self, "_c_events", [])
        return (len(ev), sum(e0.elapsed_time(e1) for _, e0, e1 in ev), sum(b for b, _, _ in ev),
                getattr(self, "_t_mb", 0))

    def _gemm(self, g, stream):
        rec = getattr(self, "_t_period", 0) and self._t_count % self._t_period == 0
        if rec:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        self.check(self.lib.lgx_gemm_nt(C.byref(g), stream), "gemm_nt")
        if rec:
            e1.record()
            # algorithmic FLOP: the unpadded K of layer 1 (num_obs), not the zero-padded columns
            k = self.k_alg.get(id(g), g.K)
            self._t_events.append((g.epi, 2.0 * g.M * g.N * k * g.batch, e0, e1))

    @property
    def join_events(self):
        """"device" (lgx_event_*) or "system" (torch events): the event kind _join uses."""
        return "device" if (os.environ.get("LGX_PPO_DEV_EVENTS", "1") != "0" and self.ppo.dist is None) else "system"

    def _device_events(self):
        if getattr(self, "_dev_ev", None) is None:
            self._dev_ev = []
            for _ in range(self.L + 1):
                e = C.c_void_p()
                self.check(self.lib.lgx_event_create(C.byref(e)), "event_create")
                self._dev_ev.append(e)
        return self._dev_ev

    def _arm(self, slot):
        """Bind join `slot`'s device event to the next lgx launch (the producer's last one), so the
        join records no separate event packet on the producer stream: each record left the stream
        idle ~5 us between two kernels.  LGX_PPO_BIND=0: recorded at the join as before."""
        if self.join_events != "device" or os.environ.get("LGX_PPO_BIND", "1") == "0":
            return
        self.check(self.lib.lgx_launch_bind_event(self._device_events()[slot]), "launch_bind_event")
        self._armed = slot

    def _join(self, src, dst, slot):
        """Order `dst` after the work issued so far on `src` (slot: 0..L-1 the side stream's inputs,
        L its output).  Device-scope events (lgx_event_*: no system-scope cache write-back and
        invalidate at the record) in single-process runs unless LGX_PPO_DEV_EVENTS=0 (torch events;
        read per call for same-process A/B runs).  Data-parallel runs keep the system-scope events:
        the joins there also order the collectives' buffers, which peers write over xGMI."""
        if self.join_events == "device":
            e = self._device_events()[slot]
            armed, self._armed = getattr(self, "_armed", None), None
            # bound to the producer's last launch by _arm (no record packet on `src`), else recorded
            if armed != slot or self.lib.lgx_launch_bind_pending():
                if armed is not None:
                    self.lib.lgx_launch_bind_pending()   # (a stale binding: disarm)
                self.check(self.lib.lgx_event_record(e, C.c_void_p(src.cuda_stream)), "event_record")
            self.check(self.lib.lgx_stream_wait_event(C.c_void_p(dst.cuda_stream), e), "stream_wait_event")
        else:
            e = self._ev_in[slot] if slot < self.L else self._ev_out
            e.record(src)
            dst.wait_event(e)

    def __del__(self):
        for e in getattr(self, "_dev_ev", None) or []:
            try:
                self.lib.lgx_event_destroy(e)
            except Exception:
                pass

    def _gemm_tn(self, t, stream, torch_stream=None):
        rec = getattr(self, "_t_period", 0) and self._t_count % self._t_period == 0   # (as _gemm)
        if rec:   # (events on the stream the kernel runs on)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch_stream)
        self.check(self.lib.lgx_gemm_tn(C.byref(t), stream), "gemm_tn")
        if rec:
            e1.record(torch_stream)
            self._t_events.append(("tn", 2.0 * t.M * t.R * t.Cc * t.batch, e0, e1))

    def gemm_timings(self):
        """{epilogue: (launches, total ms, total algorithmic FLOP, timed minibatches)} of the timed
        launches."""
        torch.cuda.synchronize()
        out = {}
        for epi, flop, e0, e1 in getattr(self, "_t_events", []):
            n, ms, f, _ = out.get(epi, (0, 0.0, 0.0, 0))
            out[epi] = (n + 1, ms + e0.elapsed_time(e1), f + flop, self._t_mb)
        return out

    @torch.no_grad()
    def _minibatch(self, idx, obs, cobs, args, stream, apply=True, xs=None):
        with self.tuned:     # TunableOp table on for the library GEMMs of this minibatch only
            self._minibatch_body(idx, obs, cobs, args, stream, apply, xs)

    def _minibatch_body(self, idx, obs, cobs, args, stream, apply=True, xs=None):
        """One minibatch: rows `idx` of the storage; `xs` = their padded layer-1 inputs already
        gathered (slices of _gather_all's buffers), None = gather here."""
        lib, chk = self.lib, self.check
        ppo = self.ppo
        M, S, h, L, A = self.M, self.S, self.hidden, self.L, self.A
        if getattr(self, "_t_period", 0):
            self._t_mb += self._t_count % self._t_period == 0
            self._t_count += 1
        fused = self.lgx_gemm
        X = Xc = self.X
        if fused:
            if not self._mirrors_valid:   # (afterwards lgx_adam_clip_mirror keeps the copies current)
                if self.split:
                    chk(lib.lgx_split_bf16(self.copy_jobs, len(self.copy_jobs), stream), "split_bf16")
                else:
                    chk(lib.lgx_copy2d(self.copy_jobs, len(self.copy_jobs), stream), "copy2d")
                self._mirrors_valid = True
            if xs is None:
                chk(lib.lgx_ppo_gather_rows_padded(_vp(obs), _vp(self.Xp), _vp(idx), M, obs.shape[1], self.Kp,
                                                   stream), "gather")
                if cobs is not None:
                    chk(lib.lgx_ppo_gather_rows_padded(_vp(cobs), _vp(self.Xcp), _vp(idx), M, cobs.shape[1],
                                                       self.Kcp, stream), "gather")
                xp, xcp = self.Xp, self.Xcp
            else:
                xp, xcp = xs[0], xs[1]
                if len(xs) > 2:                 # [2, M, Kp]: net 0's copy feeds the forward
                    xp = xs[0][0]
            X = Xc = xp[:, :self.num_obs]
            if cobs is not None or self.recurrent:
                Xc = xcp[:, :self.num_cobs]
            for g, src in zip(self.gemm_fwd[0], self.fwd0_src):
                g.A = (xp if src == "x" or xcp is None else xcp).data_ptr()
        else:
            chk(lib.lgx_ppo_gather_rows(_vp(obs), _vp(self.X), _vp(idx), M, obs.shape[1], stream), "gather")
            if cobs is not None:
                chk(lib.lgx_ppo_gather_rows(_vp(cobs), _vp(self.Xc), _vp(idx), M, cobs.shape[1], stream), "gather")
                Xc = self.Xc
        # ---- forward
        wa, wc = self.W[0]
        fp = self.flat_p
        if fused:
            for g in self.gemm_fwd[0]:
                self._gemm(g, stream)
            for k in range(1, L):
                if k in self.lgx_fwd_layers:
                    self._gemm(self.gemm_fwd[k], stream)
                else:
                    torch.bmm(self.Y[k - 1], self.W[k].transpose(1, 2), out=self.Y[k])
                    chk(lib.lgx_bias_act(_vp(self.Y[k]), C.c_void_p(fp.data_ptr() + 4 * self.bo[k]), M, h[k], 2, 1,
                                         stream), "bias")
        else:
            if cobs is None:   # shared input: one batched GEMM over {actor, critic} with a stride-0 input
                torch.bmm(X.unsqueeze(0).expand(2, M, self.num_obs), self.W1s.transpose(1, 2), out=self.Y[0])
            else:
                torch.mm(X, wa.t(), out=self.Y[0][0])
                torch.mm(Xc, wc.t(), out=self.Y[0][1])
            chk(lib.lgx_bias_act(_vp(self.Y[0]), C.c_void_p(fp.data_ptr() + 4 * self.bo[0]), M, h[0], 2, 1, stream),
                "bias")
            for k in range(1, L):
                torch.bmm(self.Y[k - 1], self.W[k].transpose(1, 2), out=self.Y[k])
                chk(lib.lgx_bias_act(_vp(self.Y[k]), C.c_void_p(fp.data_ptr() + 4 * self.bo[k]), M, h[k], 2, 1,
                                     stream), "bias")
        wha, whc = self.W[L]
        if not self.head_in_loss:
            torch.mm(self.Y[L - 1][0], wha.t(), out=self.MU)
            torch.mm(self.Y[L - 1][1], whc.t(), out=self.V)
        # ---- loss, gradient at the heads, KL -> adaptive learning rate
        args.idx = idx.data_ptr()
        adaptive = ppo.desired_kl is not None and ppo.schedule == "adaptive"   # (single process: in the loss finalize)
        side_on = self.tn and os.environ.get("LGX_PPO_DW_SIDE", "1") != "0"
        if self.loss_bwd:
            # loss + output-layer backward in one launch (dZ3 over Y[L-1]); finalize in the reduction
            if side_on and (L - 1) in self.gemm_dw:
                self._arm(L - 1)   # (the first join's producer)
            chk(lib.lgx_ppo_loss_bwd(C.byref(args), _vp(self.head_parts), stream), "lgx_ppo_loss_bwd")
        else:
            chk(lib.lgx_ppo_loss(C.byref(args), stream), "lgx_ppo_loss")
            # ---- backward (+ the loss finalize on one extra workgroup of the same launch)
            chk(lib.lgx_head_bwd_finalize(C.byref(args), _vp(self.dMU), _vp(self.dV), _vp(wha), _vp(whc),
                                          _vp(self.Y[L - 1]), M, A, h[-1], _vp(self.head_parts), stream), "head_bwd")
        dZ = self.Y[L - 1]                           # dZ of the last hidden layer (in place)
        # dW_k (lgx_gemm_tn) of the hidden layers on a second stream, concurrent with dA_k on this
        # one (both only read dZ_k and Y_{k-1}): the weight-gradient tiles fill the CUs that the
        # dA launch's last round leaves idle (measured 19.3 -> 19.0 ms per iteration);
        # LGX_PPO_DW_SIDE=0 keeps every launch on one stream
        side_used = False
        for k in range(L - 1, 0, -1):
            # dW_k = dZ_k^T Y_{k-1}, split-K over S row slices (partials reduced below); each dW on
            # the side stream right after its own join (dW3 held back to dA3's join, so that it
            # shares one join with dW2: 10.47 -> 10.82 ms per update - the dA3 / dW3 overlap is worth
            # more than the join)
            Sl = self.Sk[k]
            if k in self.gemm_dw and side_on:
                if getattr(self, "_side", None) is None:
                    self._side = torch.cuda.Stream(self.dev)
                    self._ev_in = [torch.cuda.Event() for _ in range(L)]
                    self._ev_out = torch.cuda.Event()
                main = torch.cuda.current_stream(self.dev)
                self._join(main, self._side, k)
                for t in self.gemm_dw[k]:
                    self._gemm_tn(t, C.c_void_p(self._side.cuda_stream), self._side)
                side_used = True
            elif k in self.gemm_dw:
                for t in self.gemm_dw[k]:
                    self._gemm_tn(t, stream)
            else:
                torch.bmm(dZ.view(2 * Sl, M // Sl, h[k]).transpose(1, 2),
                          self.Y[k - 1].view(2 * Sl, M // Sl, h[k - 1]), out=self.P[k])
            if fused:
                if side_on and k - 1 >= 1 and (k - 1) in self.gemm_dw:
                    self._arm(k - 1)   # (the next join's producer: this dA launch)
                self._gemm(self.gemm_bwd[k], stream)
            else:
                torch.bmm(dZ, self.W[k], out=self.D[k - 1])
                chk(lib.lgx_elu_bwd_colsum(_vp(self.D[k - 1]), _vp(self.Y[k - 1]), M, h[k - 1], 2,
                                           _vp(self.col_parts[k - 1]), stream), "elu_bwd")
            dZ = self.D[k - 1]
        early = (side_used and self.loss_bwd and len(self.jobs_rest) > 0
                 and os.environ.get("LGX_PPO_EARLY_REDUCE", "1") != "0")
        use_sq = self.fused_sq and apply and ppo.dist is None
        step_p = _vp(self.optimizer.step_dev) if use_sq else None
        sq = self.sq_parts.data_ptr() if use_sq else 0
        nsq = 0
        if early:
            # every gradient block but dW1's is complete once dA_1 (this stream) and the side
            # stream's dW GEMMs are: reduce them (+ the loss finalize) on the side stream while dW1
            # runs here - the memory-bound reduction next to the MFMA-bound GEMM
            if not self.rest_on_side:   # (skipping the join when possible: 10.478 -> 10.468 ms per update)
                self._join(torch.cuda.current_stream(self.dev), self._side, 0)
            self._arm(L)   # (the final join's producer: the side stream's last launch)
            if use_sq:
                chk(lib.lgx_reduce_slices_sq(self.jobs_rest, len(self.jobs_rest), C.byref(args), C.c_void_p(sq), step_p,
                                             C.c_void_p(self._side.cuda_stream)), "reduce")
            else:
                chk(lib.lgx_reduce_slices_finalize(self.jobs_rest, len(self.jobs_rest), C.byref(args),
                                                   C.c_void_p(self._side.cuda_stream)), "reduce")
        bucketed = early and apply and ppo.dist is not None and not self.recurrent
        self.bucketed = bucketed
        if bucketed:
            # data-parallel: the first gradient bucket (every block after dW1's in the layer-major
            # flat layout + the KL slot) is all-reduced from the side stream as soon as it is
            # reduced, concurrent with dW1's GEMM here; dW1's bucket follows below (one
            # communicator: the collectives run in issue order on every rank)
            with torch.cuda.stream(self._side):
                self.g_comm[self.n:].copy_(self.stats[0:1])
                self._all_reduce(self.g_comm[self.nW1:], self._side)
        if 0 in self.gemm_dw and fused:     # lgx_gemm_tn over the minibatch's padded input rows
            t = self.gemm_dw[0]
            t[0].B = xp.data_ptr()
            if len(t) > 1:
                t[1].B = (xcp if xcp is not None else xp).data_ptr()
            for tk in t:
                self._gemm_tn(tk, stream)
        elif xs is not None and len(xs) > 2:    # one batched GEMM: 2 networks x S row slices
            x2 = xs[2].view(2 * S, M // S, self.Kp)[:, :, :self.num_obs]
            torch.bmm(dZ.view(2 * S, M // S, h[0]).transpose(1, 2), x2, out=self.P[0].view(2 * S, h[0], self.num_obs))
        else:
            torch.bmm(dZ[0].view(S, M // S, h[0]).transpose(1, 2), X.unflatten(0, (S, M // S)), out=self.P[0][0])
            torch.bmm(dZ[1].view(S, M // S, h[0]).transpose(1, 2), Xc.unflatten(0, (S, M // S)), out=self.P[0][1])
        if side_used and not early:   # the weight gradients are complete before the reduction reads them
            self._join(self._side, torch.cuda.current_stream(self.dev), L)
        if early:   # (dW1's partials come from this stream; the side stream's blocks are joined below)
            if use_sq:
                chk(lib.lgx_reduce_slices_sq(self.jobs_dw1, len(self.jobs_dw1), None, C.c_void_p(sq + 4 * self.nsq_rest),
                                             None, stream), "reduce")
                nsq = self.nsq_rest + self.nsq_dw1
            else:
                chk(lib.lgx_reduce_slices(self.jobs_dw1, len(self.jobs_dw1), stream), "reduce")
            if bucketed:
                self._all_reduce(self.g_comm[:self.nW1], torch.cuda.current_stream(self.dev))
            self._join(self._side, torch.cuda.current_stream(self.dev), L)
        elif self.loss_bwd and use_sq:
            chk(lib.lgx_reduce_slices_sq(self.jobs, self.njobs, C.byref(args), C.c_void_p(sq), step_p, stream), "reduce")
            nsq = self.nsq_all
        elif self.loss_bwd:
            chk(lib.lgx_reduce_slices_finalize(self.jobs, self.njobs, C.byref(args), stream), "reduce")
        else:
            chk(lib.lgx_reduce_slices(self.jobs, self.njobs, stream), "reduce")
        if self.recurrent:
            self._memory_backward()
        if not apply:
            return
        grad_scale = 1.0
        if ppo.dist is not None:
            # summed gradient + summed KL (rsl_rl adapts the LR before the step, only the optimizer
            # step reads it, so adapting after the backward is equivalent): two buckets issued
            # above, or one collective here
            if not bucketed:
                self.g_comm[self.n:].copy_(self.stats[0:1])
                self._all_reduce(self.g_comm, torch.cuda.current_stream(self.dev))
            grad_scale = 1.0 / ppo.dist.get_world_size()
            if adaptive:
                chk(lib.lgx_ppo_adapt_lr(C.c_void_p(self.g_comm.data_ptr() + 4 * self.n), grad_scale,
                                         _vp(self.optimizer.lr_dev), ppo.desired_kl, stream), "adapt_lr")
        o = self.optimizer
        if fused and nsq:   # (norm from the reductions' sums of squares; step advanced there)
            chk(lib.lgx_adam_clip_mirror_sq(_vp(self.flat_p), _vp(self.flat_g), _vp(o.m), _vp(o.v), self.n, C.c_void_p(sq),
                                            nsq, ppo.max_grad_norm, _vp(o.lr_dev), _vp(o.step_dev), o.betas[0],
                                            o.betas[1], o.eps, self.copy_jobs, len(self.copy_jobs), stream), "adam")
        elif fused:   # the step also refreshes the GEMM weight copies (padded W1, transposed W2..)
            chk(lib.lgx_adam_clip_mirror(_vp(self.flat_p), _vp(self.flat_g), _vp(o.m), _vp(o.v), self.n,
                                         _vp(self.norm_parts), self.norm_parts.numel(), grad_scale, ppo.max_grad_norm,
                                         _vp(o.lr_dev), _vp(o.step_dev), o.betas[0], o.betas[1], o.eps, self.copy_jobs,
                                         len(self.copy_jobs), stream), "adam")
        else:
            chk(lib.lgx_adam_clip(_vp(self.flat_p), _vp(self.flat_g), _vp(o.m), _vp(o.v), self.n,
                                  _vp(self.norm_parts), self.norm_parts.numel(), grad_scale, ppo.max_grad_norm,
                                  _vp(o.lr_dev), _vp(o.step_dev), o.betas[0], o.betas[1], o.eps, stream), "adam")
