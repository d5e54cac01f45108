"""GPU: the hand-written f32-MFMA GEMMs of the PPO update (lgx_gemm_nt with its three epilogues,
lgx_copy2d, lgx_ppo_gather_rows_padded) against float64 torch references of the same ops.

Tolerance: exact-f32 MFMA products with f32 accumulation over K <= 512 of O(1) operands:
|C - C64| <= 2e-5 * sqrt(K) * max|C64| + 1e-6 (the k order differs from a sequential sum).
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


def _run(M, N, K, batch, epi, shared_a=False, lda_pad=0, seed=0):
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
    assert _lib().lgx_gemm_partials_floats(M, N, batch) == parts.numel()
    rc = _lib().lgx_gemm_nt(C.byref(a), _stream())
    lgxlib.check(rc, "lgx_gemm_nt")
    torch.cuda.synchronize()
    A64 = A[..., :K].double().expand(batch, M, K)
    acc = torch.bmm(A64, B.double().transpose(1, 2))
    if epi == abi.GEMM_BIAS_ELU:
        ref = torch.nn.functional.elu(acc + bias.double()[:, None, :])
    elif epi == abi.GEMM_DELU_COLSUM:
        y = Y.double()
        ref = acc * torch.where(y > 0, torch.ones_like(y), y + 1)
    else:
        ref = acc
    tol = 2e-5 * K ** 0.5 * ref.abs().max().item() + 1e-6
    err = (Cout.double() - ref).abs().max().item()
    assert err <= tol, f"M={M} N={N} K={K} batch={batch} epi={epi}: max err {err:.3e} > {tol:.3e}"
    if epi == abi.GEMM_DELU_COLSUM:
        pad = mtiles * abi.GEMM_TILE_M - M
        r = torch.nn.functional.pad(ref, (0, 0, 0, pad)).view(batch, mtiles, abi.GEMM_TILE_M, N).sum(2)
        perr = (parts.double() - r.transpose(0, 1)).abs().max().item()
        assert perr <= tol * abi.GEMM_TILE_M ** 0.5, f"colsum partials: max err {perr:.3e}"


@pytest.mark.parametrize("epi", [abi.GEMM_PLAIN, abi.GEMM_BIAS_ELU, abi.GEMM_DELU_COLSUM])
def test_gemm_epilogues(gpu, epi):
    _run(384, 256, 256, 2, epi)


@pytest.mark.parametrize("M,N,K", [(300, 128, 240), (129, 512, 16), (1, 128, 32), (4096, 256, 512)])
def test_gemm_shapes(gpu, M, N, K):
    # ragged M (row guards), odd K-step counts (240 = 15 steps, 16 = 1 step), one row
    _run(M, N, K, 2, abi.GEMM_BIAS_ELU, seed=M)
    _run(M, N, K, 1, abi.GEMM_DELU_COLSUM, seed=M + 1)


def test_gemm_shared_input_and_padded_rows(gpu):
    # layer-1 form: one input for both networks (batch stride 0), rows padded beyond K
    _run(512, 512, 240, 2, abi.GEMM_BIAS_ELU, shared_a=True, lda_pad=16)


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
