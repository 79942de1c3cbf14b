"""Row-wise top-k of the importance sampling (csrc/topk.hip radix select, used in place of
`torch.topk(uncertainty, k)[1]`, HF:m2f:689-724): the selected index SET per row equals
torch.topk's when the k-th largest value is unique in its row; with ties at the
threshold the selection is the lowest indices among them; indices come out ascending."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _check_sets(x, k):
    from visionseg import ops
    got = ops.topk_rows(x, k)
    assert got.shape == (x.shape[0], k) and got.dtype == torch.int64
    assert bool((got[:, 1:] > got[:, :-1]).all()), "indices must be strictly ascending"
    ref = torch.topk(x, k, dim=1)[1].sort(1)[0]
    return got, ref


@pytest.mark.parametrize("rows,n,k", [(1, 1, 1), (3, 100, 1), (5, 257, 257), (7, 1000, 333),
                                      (64, 37632, 9408), (4000, 12544, 9408 // 3), (2, 3 * 12544, 3 * 12544 - 1),
                                      (3, 50001, 20000), (2, 65536, 7)])
def test_topk_rows_distinct(rows, n, k):
    g = torch.Generator(device=DEV).manual_seed(rows * 7 + n)
    # distinct values of both signs (a permutation of ranks, shifted and scaled)
    x = (torch.rand(rows, n, device=DEV, generator=g).argsort(1).float() - n / 2) * 0.37
    got, ref = _check_sets(x, k)
    assert torch.equal(got, ref)


def test_topk_rows_uncertainty_signs():
    """-|logit| values (all <= 0, with exact zeros and -0.0) and mixed signs / infinities."""
    g = torch.Generator(device=DEV).manual_seed(3)
    x = -torch.abs(torch.randn(33, 5000, device=DEV, generator=g))
    x[:, ::97] = 0.0
    got, ref = _check_sets(x, 1200)
    assert torch.equal(torch.take_along_dim(x, got, 1).sort(1)[0], torch.take_along_dim(x, ref, 1).sort(1)[0])
    y = torch.randn(9, 3001, device=DEV, generator=g)
    y[0, 5] = float("inf")
    y[1, 7] = float("-inf")
    y[2, :100] = float("inf")
    got, ref = _check_sets(y, 150)
    assert torch.equal(got, ref)


def test_topk_rows_ties_take_lowest_indices():
    x = torch.zeros(4, 1000, device=DEV)
    x[:, 500:510] = 1.0              # 10 clearly largest, then 990 tied zeros
    got = __import__("visionseg").ops.topk_rows(x, 50)
    exp = torch.cat([torch.arange(40), torch.arange(500, 510)]).sort()[0].to(DEV)
    assert torch.equal(got, exp.expand(4, -1))
    xg = torch.zeros(2, 45000, device=DEV)         # the global-memory variant (row > LDS)
    xg[:, 40000:40010] = 1.0
    got = __import__("visionseg").ops.topk_rows(xg, 50)
    assert torch.equal(got, exp.expand(2, -1).where(exp < 500, exp + 39500))
    q = torch.randint(0, 4, (6, 7777), device=DEV).float()   # heavy ties everywhere
    got = __import__("visionseg").ops.topk_rows(q, 3000)
    vals = torch.take_along_dim(q, got, 1).sort(1, descending=True)[0]
    assert torch.equal(vals, torch.topk(q, 3000, dim=1)[0])
    thr = vals[:, -1:]
    # among the threshold ties, the chosen ones are the lowest positions
    for r in range(6):
        eq = (q[r] == thr[r]).nonzero().flatten()
        chosen = got[r][q[r, got[r]] == thr[r]]
        assert torch.equal(chosen, eq[:chosen.numel()])


def test_topk_rows_graph_capture():
    from visionseg import ops
    x = torch.rand(4000, 3000, device=DEV).argsort(1).float()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.topk_rows(x, 700)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = ops.topk_rows(x, 700)
    x.copy_(-torch.rand_like(x).argsort(1).float())
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, torch.topk(x, 700, dim=1)[1].sort(1)[0])
