"""33..64-row decode GEMMs with the split-K reduction inside the tile kernel (gemm.hip
splitk_fused_epilogue: the last split of each tile sums every split's partial and applies the
epilogue) vs the two-launch form (partials, then the reduce kernel): the same bits for NONE / BIAS /
SWIGLU / RESID with and without a deferred row norm, the row sums of squares equal to the fp32
sums of the new rows, and the tile counters left zero (graph replays depend on it)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402

DEV = torch.device("cuda", 0)


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


class _Mode:
    def __init__(self, fused):
        self.fused = fused

    def __enter__(self):
        self.old = (K.SPLITK_FUSED, R.SPLITK_FUSED)
        K.SPLITK_FUSED = R.SPLITK_FUSED = self.fused

    def __exit__(self, *exc):
        K.SPLITK_FUSED, R.SPLITK_FUSED = self.old


@pytest.mark.parametrize("M", [33, 48, 64])
@pytest.mark.parametrize("N,Kd,epi", [(9216, 3072, K.EPI_NONE), (16384, 3072, K.EPI_SWIGLU), (3072, 8192, K.EPI_RESID),
                                      (3072, 3072, K.EPI_BIAS), (4096, 14336, K.EPI_RESID)])
@pytest.mark.parametrize("norm", [False, True])
def test_fused_splitk_equals_two_launch(M, N, Kd, epi, norm):
    if norm and epi == K.EPI_RESID:
        pytest.skip("a residual producer never takes a deferred norm (gemm_dk contract)")
    torch.manual_seed(M * 7 + N + Kd)
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi == K.EPI_BIAS else None
    r = _rand(M, N) if epi == K.EPI_RESID else None
    ssq_in = None
    if norm:
        ssq_in = torch.rand(8 * 64, device=DEV) * Kd
        ssq_in = (ssq_in, 8, 1e-5)
    outs = {}
    for fused in (True, False):
        with _Mode(fused):
            x = r.clone() if r is not None else None
            ssq = torch.zeros(512 * 64, dtype=torch.float32, device=DEV) if epi == K.EPI_RESID else None
            o = K.gemm_dk(a, w, epi=epi, bias=bias, resid=x, out=x, norm_in=ssq_in,
                          ssq_out=ssq if epi == K.EPI_RESID and N % 512 == 0 else None)
            torch.cuda.synchronize()
            outs[fused] = (o.clone(), ssq, K.dk_parts(N, M))
    assert torch.equal(outs[True][0], outs[False][0]), (outs[True][0].float() - outs[False][0].float()).abs().max()
    if epi == K.EPI_RESID and N % 512 == 0:
        for fused in (True, False):
            o, ssq, parts = outs[fused]
            sums = ssq.view(-1, 64)[:parts, :M].sum(0)
            torch.testing.assert_close(sums, o.float().pow(2).sum(-1), atol=1e-2 * N, rtol=1e-3)
        assert outs[True][2] == N // 128 and outs[False][2] == N // 512
    assert int(K._splitk_cnt(DEV).abs().sum()) == 0  # every tile counter back to zero


def test_fused_splitk_graph_replay_and_reference():
    """Captured in a HIP graph and replayed with new inputs (counters must reset every launch); the
    result matches the fp32 reference."""
    torch.manual_seed(3)
    M, N, Kd = 64, 9216, 3072
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        K.gemm_dk(a, w, out=out)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        K.gemm_dk(a, w, out=out)
    for rep in range(3):
        a.copy_(_rand(M, Kd))
        g.replay()
        torch.cuda.synchronize()
        ref = R.gemm(a, w)
        assert (out.float() - ref.float()).abs().max() < 0.05, rep
    assert int(K._splitk_cnt(DEV).abs().sum()) == 0
