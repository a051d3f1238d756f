"""BatchNorm finalize (adr_bn_finalize / adr_bn_bwd_finalize): the per-channel reduction of the [P][2][C] partial
rows every BN producer writes (reference nn/modules/conv.py:36-54 BatchNorm2d in train mode: batch mean and biased
variance, running stats with the unbiased variance; backward dgamma = sum g * xhat, dbeta = sum g and the
coefficients of dx = A g + B x + C). Long finalizes (P > 4096 rows, > 2048 at C >= 256) first pre-sum blocks of
rows over the whole chip (fin_presum_kernel); both forms must agree with an fp64 restatement of the same partials,
and with each other to fp32 rounding, across the P / C shapes of the n-scale step (P 64 - 25 600, C 8 - 256) and
ragged row counts."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(64, 256), (2048, 64), (3200, 128), (3200, 256), (4097, 32), (12800, 8), (25600, 16), (10240, 16),
          (7777, 48)]


def _fwd(part, P, C, count, monkeypatch, mode):
    from adrefine import kernels as K
    from adrefine.native import lib
    monkeypatch.setenv("ADR_FIN_PRESUM", mode)
    dev = part.device
    g = torch.linspace(0.5, 1.5, C, device=dev)
    b = torch.linspace(-0.2, 0.2, C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    sc, sh, mu, rs = (torch.full((C,), float("nan"), device=dev) for _ in range(4))
    fp = K.fptr
    lib.adr_bn_finalize(fp(part), P, C, count, fp(g), fp(b), fp(rm), fp(rv), 0.03, 1e-3, 1, fp(sc), fp(sh), fp(mu),
                        fp(rs), K.stream())
    torch.cuda.synchronize()
    return dict(scale=sc, shift=sh, mean=mu, rstd=rs, rm=rm, rv=rv, g=g, b=b)


def _bwd(part, P, C, count, mean, rstd, monkeypatch, mode):
    from adrefine import kernels as K
    from adrefine.native import lib
    monkeypatch.setenv("ADR_FIN_PRESUM", mode)
    dev = part.device
    g = torch.linspace(0.5, 1.5, C, device=dev)
    dg, db, A, B, Cc = (torch.full((C,), float("nan"), device=dev) for _ in range(5))
    fp = K.fptr
    lib.adr_bn_bwd_finalize(fp(part), P, C, count, fp(mean), fp(rstd), fp(g), fp(dg), fp(db), fp(A), fp(B), fp(Cc), 1,
                            0, K.stream())
    torch.cuda.synchronize()
    return dict(dgamma=dg, dbeta=db, A=A, B=B, C=Cc, g=g)


@pytest.mark.parametrize("P,C", SHAPES)
def test_bn_finalize_long_rows(monkeypatch, P, C):
    torch.manual_seed(P + C)
    rows = 128.0
    x1 = torch.randn(P, C, device="cuda") * 3 + 1.5               # per-row sums of 128 values
    x2 = x1 * x1 / rows + torch.rand(P, C, device="cuda") * rows  # sums of squares (>= sum^2 / n)
    part = torch.stack([x1, x2], 1).contiguous().view(-1)
    count = float(P * rows)
    out = {m: _fwd(part, P, C, count, monkeypatch, m) for m in ("0", "1")}
    s1, s2 = x1.double().sum(0), x2.double().sum(0)
    mean = s1 / count
    var = (s2 / count - mean * mean).clamp_min(0)
    rstd = 1.0 / torch.sqrt(var + 1e-3)
    for m, o in out.items():
        assert torch.isfinite(o["scale"]).all(), m
        torch.testing.assert_close(o["mean"].double(), mean, rtol=2e-6, atol=1e-7)
        torch.testing.assert_close(o["rstd"].double(), rstd, rtol=2e-6, atol=0)
        torch.testing.assert_close(o["scale"].double(), o["g"].double() * rstd, rtol=2e-6, atol=0)
        unb = var * count / (count - 1)
        torch.testing.assert_close(o["rv"].double(), 0.97 + 0.03 * unb, rtol=2e-6, atol=1e-7)
    for k in ("scale", "shift", "mean", "rstd"):
        torch.testing.assert_close(out["0"][k], out["1"][k], rtol=1e-6, atol=1e-7)

    # backward: partial rows (sum g, sum g * x) against the forward's mean / rstd
    gsum = torch.randn(P, C, device="cuda") * 2
    gx = torch.randn(P, C, device="cuda") * 5
    bpart = torch.stack([gsum, gx], 1).contiguous().view(-1)
    mu, rs = out["1"]["mean"], out["1"]["rstd"]
    bo = {m: _bwd(bpart, P, C, count, mu, rs, monkeypatch, m) for m in ("0", "1")}
    sg, sgxr = gsum.double().sum(0), gx.double().sum(0)
    sgx = (sgxr - mu.double() * sg) * rs.double()
    for m, o in bo.items():
        torch.testing.assert_close(o["dbeta"].double(), sg, rtol=1e-5, atol=1e-3)
        torch.testing.assert_close(o["dgamma"].double(), sgx, rtol=1e-5, atol=1e-3)
    # the sums are ~1e2 in magnitude from fp32 rows: the two orders differ by fp32 rounding of the pre-summed rows
    for k in ("dgamma", "dbeta"):
        torch.testing.assert_close(bo["0"][k], bo["1"][k], rtol=1e-5, atol=1e-4)
    for k in ("A", "B", "C"):
        torch.testing.assert_close(bo["0"][k], bo["1"][k], rtol=1e-5, atol=1e-9)


def test_bn_finalize_presum_deterministic(monkeypatch):
    """Two finalizes of the same long partials: bitwise equal (fixed split and order)."""
    torch.manual_seed(0)
    P, C = 12800, 32
    part = torch.randn(P * 2 * C, device="cuda").abs()
    a = _fwd(part, P, C, P * 128.0, monkeypatch, "1")
    b = _fwd(part, P, C, P * 128.0, monkeypatch, "1")
    for k in ("scale", "shift", "mean", "rstd"):
        assert torch.equal(a[k], b[k])
