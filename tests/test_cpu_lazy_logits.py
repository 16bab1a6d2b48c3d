"""LazyLogits (pgmi/lazy_logits.py) indexing and materialisation semantics, on CPU with a stand-in
lm_head (the GPU tests check the real pgmi_lm_head against the reference's all-row logits)."""
import torch

from pgmi.lazy_logits import LazyLogits

B, L, H, V = 2, 5, 8, 11


def _make():
    g = torch.Generator().manual_seed(0)
    hidden = torch.randn(B * L, H, generator=g)
    E = torch.randn(V, H, generator=g)
    calls = []

    def lm_head(x):
        calls.append(x.shape[0])
        return x @ E.T

    full = (hidden @ E.T).view(B, L, V)
    # the eager last row differs slightly (GEMV vs GEMM accumulation order)
    last = full[:, -1:, :] + 1e-3
    return LazyLogits(last.clone(), hidden, lm_head, B, L), full, last, calls


def test_last_row_reads_do_not_materialize():
    x, full, last, calls = _make()
    assert x.shape == (B, L, V) and x.size(1) == L and x.dim() == 3 and x.dtype == torch.float32
    for got in (x[:, -1, :], x[:, -1], x[..., -1, :], x[:, L - 1, :]):
        assert torch.equal(got, last[:, 0])
    assert torch.equal(x[1, -1], last[1, 0])
    assert torch.equal(x[:, -1, 3:7], last[:, 0, 3:7])
    assert not x.is_materialized and calls == []


def test_other_reads_materialize_once_with_the_eager_last_row():
    x, full, last, calls = _make()
    assert torch.equal(x[:, 0, :], full[:, 0])
    assert torch.equal(x[:, :-1], full[:, :-1])
    m = x.materialize()
    assert torch.equal(m[:, :-1], full[:, :-1]) and torch.equal(m[:, -1:], last)
    assert torch.equal(x[:, -1, :], last[:, 0])
    assert calls == [B * L]


def test_torch_functions_methods_and_operators():
    x, full, last, calls = _make()
    ref = full.clone()
    ref[:, -1:] = last
    assert torch.equal(torch.argmax(x, dim=-1), ref.argmax(-1))
    assert torch.equal(torch.softmax(x, -1), torch.softmax(ref, -1))
    assert torch.equal(x.float(), ref)
    assert torch.equal(x * 2, ref * 2) and torch.equal(1 - x, 1 - ref)
    assert torch.equal(x[..., :-1, :].contiguous(), ref[:, :-1])
    assert calls == [B * L]


def test_inference_loop_pattern():
    """inference.py:63-68: next_token_logits = logits[:, -1, :]; argmax(dim=-1, keepdim=True)."""
    x, full, last, calls = _make()
    nt = torch.argmax(x[:, -1, :], dim=-1, keepdim=True)
    assert torch.equal(nt, last[:, 0].argmax(-1, keepdim=True))
    assert calls == []


def test_in_place_ops_after_materialization_reach_every_read():
    """A real (B, L, V) tensor has one storage: in-place ops on it, or writes through a last-row
    view, must be seen by later last-row reads."""
    x, full, last, calls = _make()
    x.materialize()
    x.div_(2.0)                                   # tensor method through __getattr__, in place
    assert torch.equal(x[:, -1, :], last[:, 0] / 2)
    v = x[:, -1, :]
    v.mul_(4.0)                                   # write through a last-row view
    assert torch.equal(x.materialize()[:, -1], last[:, 0] * 2)
    assert torch.equal(x[:, 0, :], full[:, 0] / 2)
    assert calls == [B * L]


def test_item_assignment_materializes():
    x, full, last, calls = _make()
    x[:, -1, :] = 0.0
    assert x.is_materialized and calls == [B * L]
    assert torch.equal(x[:, -1, :], torch.zeros(B, V))
    assert torch.equal(x[:, 0, :], full[:, 0])
    x[:, 1, 2] /= 4
    assert torch.equal(x[:, 1, 2], full[:, 1, 2] / 4)
