"""GPU: the hand-written GEMMs of the PPO update (lgx_gemm_nt with its three epilogues, both
product algorithms: exact f32 MFMA and the split-bf16 evaluation; lgx_copy2d,
lgx_ppo_gather_rows_padded) against float64 torch references of the same ops.

Tolerance: f32-accurate products with f32 accumulation over K <= 512 of O(1) operands:
|C - C64| <= 2e-5 * sqrt(K) * max|C64| + 1e-6 (the k order differs from a sequential sum).
test_split_bf16_is_f32_accurate additionally bounds the split-bf16 error by the exact-f32
MFMA's own error on the same data (max and mean, x1.25).
"""
import ctypes as C

import pytest
import torch

from legged_gym_amd.sim import abi
from legged_gym_amd.sim import lib as lgxlib

pytestmark = pytest.mark.gpu


def _lib():
    return lgxlib.load()


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


ALGOS = [abi.GEMM_ALGO_F32, abi.GEMM_ALGO_SPLIT_BF16]


def _presplit(B, transpose=False):
    """lgx_split_bf16 of a [batch, rows, cols] f32 operand (transpose: of its [cols, rows] view)."""
    batch, rows, cols = B.shape
    nout, kout = (cols, rows) if transpose else (rows, cols)
    ld = _lib().lgx_split_bf16_elems(1, kout)
    Bs = torch.full((batch * nout * ld,), -1, dtype=torch.int16, device=B.device)
    j = abi.LgxCopy2dJob()
    j.src, j.dst = B.data_ptr(), Bs.data_ptr()
    j.src_ld, j.src_bs, j.dst_ld, j.dst_bs = cols, rows * cols, ld, nout * ld
    j.rows, j.cols, j.batch, j.transpose = rows, cols, batch, int(transpose)
    lgxlib.check(_lib().lgx_split_bf16((abi.LgxCopy2dJob * 1)(j), 1, _stream()), "split_bf16")
    return Bs


def _limb_index(nout, kout, device):
    """x3_limb_off (lgx_internal.h): [3, nout, kb*32] offsets of the tiled pre-split layout."""
    kb = -(-kout // 32)
    n = torch.arange(nout, device=device)[:, None]
    k = torch.arange(kb * 32, device=device)[None, :]
    nn, kk = n & 127, k & 31
    base = (n >> 7) * kb + (k >> 5)
    inner = nn * 32 + (((kk >> 3) ^ ((nn >> 2) & 3)) << 3) + (kk & 7)
    return torch.stack([(base * 3 + l) * 4096 + inner for l in range(3)])


def _limbs(Bs, batch, nout, kout):
    """[batch, 3, nout, kb*32] limbs as float64 from the tiled pre-split layout."""
    ld = _lib().lgx_split_bf16_elems(1, kout)
    idx = _limb_index(nout, kout, Bs.device)
    u = Bs.view(batch, nout * ld)[:, idx].to(torch.int32) & 0xFFFF
    return (u << 16).view(torch.float32).double()


def _limbs_to_f32(Bs, batch, nout, kout):
    return _limbs(Bs, batch, nout, kout).sum(1)


def _run(M, N, K, batch, epi, shared_a=False, lda_pad=0, seed=0, algo=abi.GEMM_ALGO_DEFAULT, presplit=False,
         tile_rows=0):
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(seed)
    lda = K + lda_pad
    A = torch.randn(1 if shared_a else batch, M, lda, device=dev, generator=g)
    B = torch.randn(batch, N, K, device=dev, generator=g) / K ** 0.5
    bias = torch.randn(batch, N, device=dev, generator=g)
    Y = torch.nn.functional.elu(torch.randn(batch, M, N, device=dev, generator=g))
    Cout = torch.full((batch, M, N), float("nan"), device=dev)
    mtiles = -(-M // abi.GEMM_TILE_M)
    parts = torch.full((mtiles, batch, N), float("nan"), device=dev)
    a = abi.LgxGemmArgs()
    a.M, a.N, a.K, a.batch, a.epi = M, N, K, batch, epi
    a.A, a.lda, a.sa = A.data_ptr(), lda, 0 if shared_a else M * lda
    a.B, a.ldb, a.sb = B.data_ptr(), K, N * K
    a.C, a.ldc, a.sc = Cout.data_ptr(), N, M * N
    a.bias, a.Y, a.partials = bias.data_ptr(), Y.data_ptr(), parts.data_ptr()
    a.algo, a.tile_rows = algo, tile_rows
    if presplit:
        Bs = _presplit(B)
        a.Bs = Bs.data_ptr()
    assert _lib().lgx_gemm_partials_floats(M, N, batch) == parts.numel()
    rc = _lib().lgx_gemm_nt(C.byref(a), _stream())
    lgxlib.check(rc, "lgx_gemm_nt")
    torch.cuda.synchronize()
    A64 = A[..., :K].double().expand(batch, M, K)
    acc = torch.bmm(A64, B.double().transpose(1, 2))
    if epi == abi.GEMM_BIAS_ELU:
        ref = torch.nn.functional.elu(acc + bias.double()[:, None, :])
    elif epi in (abi.GEMM_DELU_COLSUM, abi.GEMM_DELU):
        y = Y.double()
        ref = acc * torch.where(y > 0, torch.ones_like(y), y + 1)
    else:
        ref = acc
    tol = 2e-5 * K ** 0.5 * ref.abs().max().item() + 1e-6
    err = (Cout.double() - ref).abs().max().item()
    assert err <= tol, f"M={M} N={N} K={K} batch={batch} epi={epi} algo={algo}: max err {err:.3e} > {tol:.3e}"
    if epi == abi.GEMM_DELU_COLSUM:
        pad = mtiles * abi.GEMM_TILE_M - M
        r = torch.nn.functional.pad(ref, (0, 0, 0, pad)).view(batch, mtiles, abi.GEMM_TILE_M, N).sum(2)
        perr = (parts.double() - r.transpose(0, 1)).abs().max().item()
        assert perr <= tol * abi.GEMM_TILE_M ** 0.5, f"colsum partials: max err {perr:.3e}"


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("epi", [abi.GEMM_PLAIN, abi.GEMM_BIAS_ELU, abi.GEMM_DELU_COLSUM])
def test_gemm_epilogues(gpu, epi, algo):
    _run(384, 256, 256, 2, epi, algo=algo)


@pytest.mark.parametrize("epi", [abi.GEMM_PLAIN, abi.GEMM_BIAS_ELU, abi.GEMM_DELU_COLSUM])
@pytest.mark.parametrize("M,N,K", [(384, 256, 256), (300, 128, 240), (1, 128, 36), (4096, 512, 512), (300, 128, 256),
                                   (1, 128, 32), (257, 384, 64), (513, 256, 128)])
def test_gemm_presplit_weights(gpu, epi, M, N, K):
    """Split-bf16 path with B pre-split by lgx_split_bf16 (the weights of the PPO GEMMs): K % 32 == 0
    runs the pipelined LDS-DMA kernel (gemm_nt_x3p_kernel; ragged M, 1 row, several N tiles),
    other K the register-staged one; both read the tiled x3_limb_off layout."""
    _run(M, N, K, 2, epi, seed=M + K, algo=abi.GEMM_ALGO_SPLIT_BF16, presplit=True)


@pytest.mark.parametrize("epi", [abi.GEMM_BIAS_ELU, abi.GEMM_DELU_COLSUM])
def test_gemm_presplit_update_shape(gpu, epi):
    """The PPO-update shape (24,576 rows, 512 outputs, K 256; layer 1 with one input shared by
    actor and critic): every persistent workgroup walks several tiles, so the load ring runs
    across tile boundaries and the bias / column-sum epilogues of consecutive tiles."""
    _run(24576, 512, 256, 2, epi, shared_a=epi == abi.GEMM_BIAS_ELU, seed=11, algo=abi.GEMM_ALGO_SPLIT_BF16,
         presplit=True)


@pytest.mark.parametrize("pm", [128, 256])
@pytest.mark.parametrize("M,N,K", [(24576, 256, 512), (4096, 512, 256), (300, 128, 256), (513, 256, 128),
                                   (1000, 128, 96), (1, 128, 32)])
def test_gemm_presplit_tile_heights(gpu, pm, M, N, K):
    """The pipelined kernel with 256-row tiles and with 128-row half tiles (chosen when they fill the
    CUs' rounds better, forced here with lgx_gemm_args.tile_rows): unrolled K 512 / 256 / 128 with the
    deferred epilogue, runtime K 96, ragged M, one row."""
    for epi in (abi.GEMM_PLAIN, abi.GEMM_BIAS_ELU):
        _run(M, N, K, 2, epi, seed=M + K + pm, algo=abi.GEMM_ALGO_SPLIT_BF16, presplit=True, tile_rows=pm)


@pytest.mark.parametrize("pm", [128, 256])
@pytest.mark.parametrize("M,N,K", [(24576, 256, 128), (24576, 512, 256), (300, 128, 256), (513, 256, 128),
                                   (1000, 128, 96), (1, 128, 32)])
def test_gemm_presplit_delu_pipelined(gpu, pm, M, N, K):
    """ELU' + bias-gradient column sums on the pipelined kernel: the epilogue at each tile's end
    with non-transposed accumulators, partial rows per 128 output rows from the waves of both tile
    heights; ragged M, one row, runtime K."""
    _run(M, N, K, 2, abi.GEMM_DELU_COLSUM, seed=M + K + pm + 1, algo=abi.GEMM_ALGO_SPLIT_BF16, presplit=True,
         tile_rows=pm)


@pytest.mark.parametrize("pm", [128, 256])
@pytest.mark.parametrize("M,N,K", [(24576, 256, 128), (24576, 512, 256), (4096, 512, 512), (300, 128, 256),
                                   (513, 256, 128), (1000, 128, 96), (1, 128, 32), (257, 384, 64)])
def test_gemm_presplit_delu_deferred(gpu, pm, M, N, K):
    """LGX_GEMM_DELU (ELU' without column sums, the backward dA of the fused update): transposed
    accumulators, the output deferred into the next tile's slots with the Y runs of every slot
    loaded one slot ahead (K 128 / 256 / 512 unrolled), at the tile's end for runtime K (96, 64, 32);
    both tile heights, ragged M, one row, several tiles per workgroup (24,576 rows)."""
    _run(M, N, K, 2, abi.GEMM_DELU, seed=M + K + pm + 3, algo=abi.GEMM_ALGO_SPLIT_BF16, presplit=True, tile_rows=pm)


def test_gemm_delu_needs_presplit(gpu):
    """LGX_GEMM_DELU exists on the pipelined split-bf16 kernel only: other paths refuse it."""
    with pytest.raises(lgxlib.LgxError):
        _run(256, 128, 64, 1, abi.GEMM_DELU, algo=abi.GEMM_ALGO_F32)
    with pytest.raises(lgxlib.LgxError):
        _run(256, 128, 64, 1, abi.GEMM_DELU, algo=abi.GEMM_ALGO_SPLIT_BF16, presplit=False)


@pytest.mark.parametrize("transpose", [False, True])
def test_split_bf16_limbs(gpu, transpose):
    """lgx_split_bf16: limbs are RNE bf16 (x0 = bf16(x), |x1| <= 2^-8|x0|, |x2| <= 2^-8|x1|),
    their sum reproduces x to 2^-26 relative, padding to the 32-k block is zero; every element
    of the buffer is written (tiled x3_limb_off layout)."""
    g = torch.Generator(device="cuda:0").manual_seed(2)
    shape = (2, 45, 256) if transpose else (2, 256, 45)
    B = torch.randn(*shape, device="cuda:0", generator=g) * torch.exp2(
        torch.randint(-20, 20, shape, device="cuda:0", generator=g).float())
    Bs = _presplit(B, transpose)
    torch.cuda.synchronize()
    assert not bool((Bs == -1).any())
    ref = (B.transpose(1, 2) if transpose else B).double()
    nout, kout = ref.shape[1], ref.shape[2]
    limbs = _limbs(Bs, 2, nout, kout)
    rec = limbs.sum(1)
    assert torch.all(rec[..., kout:] == 0)
    rec = rec[..., :kout]
    assert bool(((rec - ref).abs() <= 2.0 ** -26 * ref.abs()).all())
    x0 = limbs[:, 0, :, :kout].float()
    assert torch.equal(x0, (B.transpose(1, 2) if transpose else B).to(torch.bfloat16).float())
    assert bool((limbs[:, 1].abs() <= 2.0 ** -8 * limbs[:, 0].abs()).all())   # half a bf16 ulp
    assert bool((limbs[:, 2].abs() <= 2.0 ** -8 * limbs[:, 1].abs()).all())


def test_split_bf16_rejects_ragged_rows(gpu):
    B = torch.zeros(1, 100, 64, device="cuda:0")
    j = abi.LgxCopy2dJob()
    Bs = torch.zeros(1 << 16, dtype=torch.int16, device="cuda:0")
    j.src, j.dst = B.data_ptr(), Bs.data_ptr()
    j.src_ld, j.src_bs, j.dst_ld, j.dst_bs = 64, 6400, 192, 100 * 192
    j.rows, j.cols, j.batch, j.transpose = 100, 64, 1, 0
    assert _lib().lgx_split_bf16((abi.LgxCopy2dJob * 1)(j), 1, _stream()) != 0


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("M,N,K", [(300, 128, 240), (129, 512, 16), (1, 128, 32), (4096, 256, 512), (257, 384, 36)])
def test_gemm_shapes(gpu, M, N, K, algo):
    # ragged M (row guards), odd K-step counts (240 = 15 steps, 16 = 1 step, 36 = a 4-wide tail
    # stage), one row
    _run(M, N, K, 2, abi.GEMM_BIAS_ELU, seed=M, algo=algo)
    _run(M, N, K, 1, abi.GEMM_DELU_COLSUM, seed=M + 1, algo=algo)


@pytest.mark.parametrize("algo", ALGOS)
def test_gemm_shared_input_and_padded_rows(gpu, algo):
    # layer-1 form: one input for both networks (batch stride 0), rows padded beyond K
    _run(512, 512, 240, 2, abi.GEMM_BIAS_ELU, shared_a=True, lda_pad=16, algo=algo)


def _plain(A, B, algo):
    batch, M, K = A.shape
    N = B.shape[1]
    Cout = torch.full((batch, M, N), float("nan"), device=A.device)
    a = abi.LgxGemmArgs()
    a.M, a.N, a.K, a.batch, a.epi = M, N, K, batch, abi.GEMM_PLAIN
    a.A, a.lda, a.sa = A.data_ptr(), K, M * K
    a.B, a.ldb, a.sb = B.data_ptr(), K, N * K
    a.C, a.ldc, a.sc = Cout.data_ptr(), N, M * N
    a.algo = algo
    lgxlib.check(_lib().lgx_gemm_nt(C.byref(a), _stream()), "lgx_gemm_nt")
    torch.cuda.synchronize()
    return Cout


@pytest.mark.parametrize("spread", [0, 12])
def test_split_bf16_is_f32_accurate(gpu, spread):
    """The split-bf16 products are f32-accurate: against float64, the max and mean absolute
    errors stay within 1.25x those of the exact-f32 MFMA (fmaf chain) on the same operands,
    including operands whose magnitudes spread over 2^+-spread (limb exponents follow each
    element); every element's error is within the classic f32 dot-product bound
    K * 2^-24 * sum_k |a b| (recursive summation, gamma_K)."""
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(17 + spread)
    M, N, K = 2048, 256, 512
    A = torch.randn(2, M, K, device=dev, generator=g)
    B = torch.randn(2, N, K, device=dev, generator=g)
    if spread:
        A = A * torch.exp2(torch.randint(-spread, spread + 1, A.shape, device=dev, generator=g).float())
        B = B * torch.exp2(torch.randint(-spread, spread + 1, B.shape, device=dev, generator=g).float())
    ref = torch.bmm(A.double(), B.double().transpose(1, 2))
    scale = torch.bmm(A.double().abs(), B.double().abs().transpose(1, 2))
    e32 = (_plain(A, B, abi.GEMM_ALGO_F32).double() - ref).abs()
    esp = (_plain(A, B, abi.GEMM_ALGO_SPLIT_BF16).double() - ref).abs()
    assert esp.max().item() <= 1.25 * e32.max().item(), (esp.max().item(), e32.max().item())
    assert esp.mean().item() <= 1.25 * e32.mean().item(), (esp.mean().item(), e32.mean().item())
    assert bool((esp <= K * 2.0 ** -24 * scale).all())


def _run_tn(M, S, R, Cc, batch, ldb=None, seed=0, colsum=False):
    """lgx_gemm_tn against float64: C[z][s] = A[z, slice s]^T B[z, slice s, :Cc] (and with colsum
    the per-slice column sums of A)."""
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(seed)
    ldb = ldb or Cc
    A = torch.randn(batch, M, R, device=dev, generator=g)
    B = torch.randn(batch, M, ldb, device=dev, generator=g)
    Cout = torch.full((batch, S, R, Cc), float("nan"), device=dev)
    a = abi.LgxGemmTnArgs()
    a.M, a.R, a.Cc, a.slices, a.batch = M, R, Cc, S, batch
    a.A, a.lda, a.sa = A.data_ptr(), R, M * R
    a.B, a.ldb, a.sb = B.data_ptr(), ldb, M * ldb
    a.C, a.ldc = Cout.data_ptr(), Cc
    cs = torch.full((batch, S, R), float("nan"), device=dev)
    if colsum:
        a.colsum = cs.data_ptr()
    lgxlib.check(_lib().lgx_gemm_tn(C.byref(a), _stream()), "lgx_gemm_tn")
    torch.cuda.synchronize()
    Ms = M // S
    ref = torch.einsum("zsmn,zsmc->zsnc", A.double().view(batch, S, Ms, R), B[..., :Cc].double().view(batch, S, Ms, Cc))
    tol = 2e-5 * Ms ** 0.5 * ref.abs().max().item() + 1e-6
    err = (Cout.double() - ref).abs().max().item()
    assert err <= tol, f"M={M} S={S} R={R} Cc={Cc}: max err {err:.3e} > {tol:.3e}"
    if colsum:   # f32 sums of f32 rows (4 per thread, then 8 row groups in a fixed order)
        rcs = A.double().view(batch, S, Ms, R).sum(2)
        cerr = (cs.double() - rcs).abs().max().item()
        assert cerr <= 1e-6 * Ms * A.abs().max().item(), f"colsum max err {cerr:.3e}"


@pytest.mark.parametrize("M,S,R,Cc,ldb", [(1024, 2, 128, 128, None), (2048, 4, 256, 235, 256), (96, 3, 128, 384, None),
                                          (24576, 16, 256, 512, None), (24576, 8, 512, 235, 256),
                                          (24576, 32, 128, 256, None)])
def test_gemm_tn_weight_gradients(gpu, M, S, R, Cc, ldb):
    """lgx_gemm_tn (dW = dZ^T Y over row slices, split-bf16 products, transposed LDS reads):
    small and update-sized shapes, ragged output columns (235 = num_obs, padded input rows),
    one stage per slice (96 / 3 = 32 rows), several column tiles."""
    _run_tn(M, S, R, Cc, 2, ldb=ldb, seed=M + S)


@pytest.mark.parametrize("M,S,R,Cc,ldb", [(1024, 2, 128, 128, None), (2048, 4, 256, 235, 256), (96, 3, 128, 384, None),
                                          (24576, 16, 256, 512, None), (24576, 16, 512, 235, 256),
                                          (24576, 32, 128, 256, None)])
def test_gemm_tn_column_sums(gpu, M, S, R, Cc, ldb):
    """lgx_gemm_tn's colsum (the bias gradient db = column sums of dZ, per row slice, taken from
    the staged f32 rows by the first column tile of each output row tile): one stage per slice,
    ragged output columns, several row and column tiles, both tile heights."""
    _run_tn(M, S, R, Cc, 2, ldb=ldb, seed=M + S + 7, colsum=True)


@pytest.mark.parametrize("M,S,R,Cc,ldb", [(2048, 4, 256, 235, 256), (96, 3, 128, 384, None), (24576, 16, 512, 235, 256),
                                          (24576, 32, 128, 256, None), (24576, 16, 256, 512, None)])
def test_gemm_tn_warp_specialised_equals_plain(gpu, monkeypatch, M, S, R, Cc, ldb):
    """The warp-specialised dW kernel (producer waves stage and split, consumer waves only read
    fragments and issue MFMAs; with LGX_TN_RING=0 the form for 128-row tiles) against gemm_tn_x3_kernel (LGX_TN_WS=0): the same products in
    the same order per output element, so the weight gradients are bitwise equal; the column sums
    (other per-thread row groups) within f32 rounding."""
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(M + R)
    ldb = ldb or Cc
    A = torch.randn(2, M, R, device=dev, generator=g)
    B = torch.randn(2, M, ldb, device=dev, generator=g)
    monkeypatch.setenv("LGX_TN_RING", "0")
    outs = []
    for ws in ("2", "0"):        # (2: the warp-specialised kernel at both tile heights)
        monkeypatch.setenv("LGX_TN_WS", ws)
        Cout = torch.full((2, S, R, Cc), float("nan"), device=dev)
        cs = torch.full((2, S, R), float("nan"), device=dev)
        a = abi.LgxGemmTnArgs()
        a.M, a.R, a.Cc, a.slices, a.batch = M, R, Cc, S, 2
        a.A, a.lda, a.sa = A.data_ptr(), R, M * R
        a.B, a.ldb, a.sb = B.data_ptr(), ldb, M * ldb
        a.C, a.ldc, a.colsum = Cout.data_ptr(), Cc, cs.data_ptr()
        lgxlib.check(_lib().lgx_gemm_tn(C.byref(a), _stream()), "lgx_gemm_tn")
        torch.cuda.synchronize()
        outs.append((Cout, cs))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-5 * (M // S) ** 0.5)


@pytest.mark.parametrize("M,S,R,Cc,ldb", [(2048, 4, 256, 235, 256), (96, 3, 256, 384, None), (160, 1, 256, 128, None),
                                          (24576, 16, 512, 235, 256), (24576, 32, 256, 256, None),
                                          (24576, 16, 256, 512, None)])
def test_gemm_tn_ring_equals_plain(gpu, monkeypatch, M, S, R, Cc, ldb):
    """The 256-row tiles' ring form (16-row stages in a 3-deep LDS ring, each stage's fragments read
    before the barrier that opens it; the default) against gemm_tn_x3_kernel<8> (LGX_TN_RING=0): the
    same products in the same order per output element, so the weight gradients are bitwise equal;
    the column sums (other per-thread row groups) within f32 rounding.  Slices of 32 and 160 rows:
    2 and an odd 10 ring stages."""
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(M + R + 1)
    ldb = ldb or Cc
    A = torch.randn(2, M, R, device=dev, generator=g)
    B = torch.randn(2, M, ldb, device=dev, generator=g)
    monkeypatch.setenv("LGX_TN_WS", "1")
    outs = []
    for ring in ("1", "0"):
        monkeypatch.setenv("LGX_TN_RING", ring)
        Cout = torch.full((2, S, R, Cc), float("nan"), device=dev)
        cs = torch.full((2, S, R), float("nan"), device=dev)
        a = abi.LgxGemmTnArgs()
        a.M, a.R, a.Cc, a.slices, a.batch = M, R, Cc, S, 2
        a.A, a.lda, a.sa = A.data_ptr(), R, M * R
        a.B, a.ldb, a.sb = B.data_ptr(), ldb, M * ldb
        a.C, a.ldc, a.colsum = Cout.data_ptr(), Cc, cs.data_ptr()
        lgxlib.check(_lib().lgx_gemm_tn(C.byref(a), _stream()), "lgx_gemm_tn")
        torch.cuda.synchronize()
        outs.append((Cout, cs))
    assert not torch.isnan(outs[0][0]).any()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-5 * (M // S) ** 0.5)


@pytest.mark.parametrize("M,S,R,Cc,ldb", [(2048, 4, 128, 235, 256), (96, 3, 128, 384, None), (160, 1, 384, 128, None),
                                          (24576, 32, 128, 256, None), (24576, 16, 128, 256, None)])
def test_gemm_tn_ring_128_row_tiles_equal_ws(gpu, monkeypatch, M, S, R, Cc, ldb):
    """The ring form at 128-row tiles (the default: waves of 32 x 64) against the warp-specialised
    kernel (LGX_TN_RING=0): bitwise weight gradients, column sums within f32 rounding."""
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(M + R + 3)
    ldb = ldb or Cc
    A = torch.randn(2, M, R, device=dev, generator=g)
    B = torch.randn(2, M, ldb, device=dev, generator=g)
    monkeypatch.setenv("LGX_TN_WS", "1")
    outs = []
    for ring in ("1", "0"):
        monkeypatch.setenv("LGX_TN_RING", ring)
        Cout = torch.full((2, S, R, Cc), float("nan"), device=dev)
        cs = torch.full((2, S, R), float("nan"), device=dev)
        a = abi.LgxGemmTnArgs()
        a.M, a.R, a.Cc, a.slices, a.batch = M, R, Cc, S, 2
        a.A, a.lda, a.sa = A.data_ptr(), R, M * R
        a.B, a.ldb, a.sb = B.data_ptr(), ldb, M * ldb
        a.C, a.ldc, a.colsum = Cout.data_ptr(), Cc, cs.data_ptr()
        lgxlib.check(_lib().lgx_gemm_tn(C.byref(a), _stream()), "lgx_gemm_tn")
        torch.cuda.synchronize()
        outs.append((Cout, cs))
    assert not torch.isnan(outs[0][0]).any() and not torch.isnan(outs[0][1]).any()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-5 * (M // S) ** 0.5)


def test_gemm_tn_rejects_bad_shapes(gpu):
    a = abi.LgxGemmTnArgs()
    x = torch.zeros(4096, device="cuda:0")
    a.M, a.R, a.Cc, a.slices, a.batch = 100, 128, 128, 1, 1      # slice rows % 32 != 0
    a.A = a.B = a.C = x.data_ptr()
    a.lda = a.ldb = a.ldc = 128
    assert _lib().lgx_gemm_tn(C.byref(a), _stream()) != 0
    a.M, a.R = 128, 100                                            # R % 128 != 0
    assert _lib().lgx_gemm_tn(C.byref(a), _stream()) != 0


def test_gemm_rejects_bad_shapes(gpu):
    a = abi.LgxGemmArgs()
    x = torch.zeros(64, 64, device="cuda:0")
    a.M, a.N, a.K, a.batch, a.epi = 64, 64, 64, 1, abi.GEMM_PLAIN   # N % 128 != 0
    a.A = a.B = a.C = x.data_ptr()
    a.lda = a.ldb = a.ldc = 64
    assert _lib().lgx_gemm_nt(C.byref(a), _stream()) != 0
    a.N, a.K = 128, 24                                              # K % 16 != 0
    assert _lib().lgx_gemm_nt(C.byref(a), _stream()) != 0


def test_copy2d_and_padded_gather(gpu):
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(5)
    W = torch.randn(2, 96, 70, device=dev, generator=g)
    WT = torch.zeros(2, 70, 96, device=dev)
    Wp = torch.zeros(2, 96, 80, device=dev)
    jobs = []
    for dst, tr, dst_ld in ((WT, 1, 96), (Wp, 0, 80)):
        j = abi.LgxCopy2dJob()
        j.src, j.dst = W.data_ptr(), dst.data_ptr()
        j.src_ld, j.src_bs = 70, 96 * 70
        j.dst_ld, j.dst_bs = dst_ld, dst[0].numel()
        j.rows, j.cols, j.batch, j.transpose = 96, 70, 2, tr
        jobs.append(j)
    arr = (abi.LgxCopy2dJob * 2)(*jobs)
    lgxlib.check(_lib().lgx_copy2d(arr, 2, _stream()), "copy2d")
    torch.cuda.synchronize()
    assert torch.equal(WT, W.transpose(1, 2))
    assert torch.equal(Wp[..., :70], W) and torch.all(Wp[..., 70:] == 0)
    src = torch.randn(50, 235, device=dev, generator=g)
    idx = torch.randperm(50, device=dev)[:37]
    dst = torch.full((37, 240), float("nan"), device=dev)
    lgxlib.check(_lib().lgx_ppo_gather_rows_padded(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                                   C.c_void_p(idx.data_ptr()), 37, 235, 240, _stream()), "gather")
    torch.cuda.synchronize()
    assert torch.equal(dst[:, :235], src[idx]) and torch.all(dst[:, 235:] == 0)


def test_elu_near_zero_bound(gpu):
    """lgx_elu (lgx_internal.h: exp(x) - 1 on v_exp_f32, shared by every ELU epilogue: rollout MLP,
    PPO forward GEMMs, lgx_bias_act) against float64 ELU for pre-activations concentrated near 0,
    where exp(x) - 1 cancels: the documented bound is an ABSOLUTE error of at most
    1.5e-7 (a few ulp of 1), i.e. relative error <= 1.5e-7 / |x| - tiny outputs carry large relative
    error but stay below the rounding of the O(1) sums of the next layer; x >= 0 is exact."""
    g = torch.Generator(device="cuda:0").manual_seed(4)
    mag = 10 ** (-8 + 7 * torch.rand(64 * 1024, device="cuda:0", generator=g))     # 1e-8 .. 0.1
    sign = torch.where(torch.rand(64 * 1024, device="cuda:0", generator=g) < 0.8, -1.0, 1.0)
    x = (mag * sign).view(1024, 64).contiguous()
    z = x.clone()
    zero_b = torch.zeros(64, device="cuda:0")
    lgxlib.check(_lib().lgx_bias_act(C.c_void_p(z.data_ptr()), C.c_void_p(zero_b.data_ptr()), 1024, 64, 1, 1,
                                     _stream()), "bias_act")
    torch.cuda.synchronize()
    ref = torch.nn.functional.elu(x.double())
    err = (z.double() - ref).abs()
    assert err.max().item() <= 1.5e-7, err.max().item()
    assert (err[x > 0] == 0).all()
    rel = err / ref.abs().clamp_min(1e-30)
    assert (rel <= 1.5e-7 / x.double().abs() + 1e-7).all()
    # and where the cancellation is mild (|x| >= 2^-8) the relative error is f32-level
    mild = x.abs() >= 2 ** -8
    assert rel[mild].max().item() <= 6e-5, rel[mild].max().item()


def test_device_scope_events_order_two_streams(gpu):
    """lgx_event_create / lgx_event_record / lgx_stream_wait_event (the PPO update's cross-stream
    joins, device-scope release): a consumer stream ordered after a producer stream's long chain
    of launches reads the producer's final values; destroy accepts the handle."""
    lib = _lib()
    dev = "cuda:0"
    prod, cons = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ev = C.c_void_p()
    lgxlib.check(lib.lgx_event_create(C.byref(ev)), "event_create")
    x = torch.zeros(4096, 4096, device=dev)
    w = torch.eye(4096, device=dev)
    with torch.cuda.stream(prod):
        for i in range(8):                     # long enough that an unordered reader would race it
            x = x @ w + 1.0
    lgxlib.check(lib.lgx_event_record(ev, C.c_void_p(prod.cuda_stream)), "event_record")
    lgxlib.check(lib.lgx_stream_wait_event(C.c_void_p(cons.cuda_stream), ev), "stream_wait_event")
    with torch.cuda.stream(cons):
        y = x.sum()
    torch.cuda.synchronize()
    assert y.item() == pytest.approx(8.0 * 4096 * 4096)
    assert lib.lgx_event_destroy(ev) == 0
    assert lib.lgx_event_record(None, None) != 0      # null event: error status, no crash
