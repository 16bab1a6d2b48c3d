"""Prefill logits computed lazily (SURVEY.md sec.7 hard part 3).

The reference's GemmaForCausalLM returns logits for EVERY prefill position: (B, L, 257216) fp32,
288 x 257216 x 4 B = 296 MB and a 303 GFLOP GEMM at 224 px (modeling_gemma.py:417-418), while
its callers read only the last row (inference.py:63, ablation_study_fixed.py:226).  LazyLogits
stands in for that tensor: the last row is computed eagerly by the lm_head GEMV (with the final
RMSNorm fused), the final-normed hidden rows are kept (B*L x 2048 bf16, 1.2 MB), and the full
tensor is materialised by pgmi_lm_head -- the same GEMM the eager all-row path runs -- the first
time anything other than the last row is read.  The last row of the materialised tensor is the
eager one, so every read sees one consistent tensor.

Reads of the last position (`x[:, -1, :]`, `x[:, -1]`, `x[..., -1, :]`, `x[0, L-1]`) never
materialise.  Everything else -- other indices, item assignment, torch functions
(`torch.argmax(x)`), tensor methods and operators, in-place ones included -- materialises once and
then acts on the real (B, L, V) tensor; every later read, last row included, indexes that tensor.
LazyLogits is not a torch.Tensor subclass (`isinstance(x, torch.Tensor)` is False); the
drop-in model's `pgmi_prefill_logits = "all"` returns a plain tensor.  One difference from a real
tensor remains: a last-row view taken BEFORE materialisation is a view of the eager row, not of
the later full tensor.
"""
from __future__ import annotations

import torch


class LazyLogits:
    def __init__(self, last: torch.Tensor, hidden: torch.Tensor, lm_head, B: int, L: int):
        """last: (B, 1, V) fp32 logits of position L-1; hidden: (B*L, H) final-normed rows;
        lm_head: rows -> (rows, V) fp32 (Engine.lm_head)."""
        self._last, self._hidden, self._lm_head = last, hidden, lm_head
        self._B, self._L, self._V = B, L, last.shape[-1]
        self._full = None

    # ---- tensor metadata (no materialisation)
    @property
    def shape(self) -> torch.Size:
        return torch.Size((self._B, self._L, self._V))

    @property
    def dtype(self):
        return self._last.dtype

    @property
    def device(self):
        return self._last.device

    @property
    def ndim(self) -> int:
        return 3

    @property
    def is_materialized(self) -> bool:
        return self._full is not None

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim]

    def dim(self) -> int:
        return 3

    def __len__(self) -> int:
        return self._B

    def __repr__(self) -> str:
        state = "materialized" if self._full is not None else "last row only"
        return f"LazyLogits(shape={tuple(self.shape)}, dtype={self.dtype}, device={self.device}, {state})"

    # ---- materialisation
    def materialize(self) -> torch.Tensor:
        if self._full is None:
            full = self._lm_head(self._hidden).view(self._B, self._L, self._V)
            full[:, -1:, :].copy_(self._last)  # one tensor: the eager last row wins
            self._full = full
            # from here on the last row IS a view of the full tensor, so in-place ops on either
            # (logits.div_(t), logits[:, -1, :] /= t) are seen by every later read
            self._last = full[:, -1:, :]
            self._hidden = None
        return self._full

    def _last_row_index(self, idx):
        """idx selecting within the last position only -> the equivalent index into (B, 1, V)."""
        if not isinstance(idx, tuple):
            return None
        if any(i is Ellipsis for i in idx):
            k = [j for j, i in enumerate(idx) if i is Ellipsis][0]
            fill = 3 - (len(idx) - 1)
            if fill < 0:
                return None
            idx = idx[:k] + (slice(None),) * fill + idx[k + 1:]
        if len(idx) < 2 or any(i is None for i in idx):
            return None
        p = idx[1]
        if isinstance(p, bool) or not isinstance(p, int) or p not in (-1, self._L - 1):
            return None
        return (idx[0], 0) + tuple(idx[2:])

    def __getitem__(self, idx):
        if self._full is not None:
            return self._full[idx]
        li = self._last_row_index(idx)
        if li is not None:
            return self._last[li]
        return self.materialize()[idx]

    def __setitem__(self, idx, value):
        """Item assignment acts on the real tensor (materialises first, as a (B, L, V) tensor
        would hold every row)."""
        if isinstance(value, LazyLogits):
            value = value.materialize()
        self.materialize()[idx] = value

    # ---- everything else acts on the materialised tensor
    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        def real(a):
            if isinstance(a, LazyLogits):
                return a.materialize()
            if isinstance(a, (list, tuple)):
                return type(a)(real(x) for x in a)
            return a
        return func(*real(args), **{k: real(v) for k, v in (kwargs or {}).items()})

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.materialize(), name)

    def __array__(self, dtype=None):
        a = self.materialize().cpu().numpy()
        return a if dtype is None else a.astype(dtype)


def _binop(name):
    def f(self, *args):
        return getattr(self.materialize(), name)(*[a.materialize() if isinstance(a, LazyLogits) else a for a in args])
    f.__name__ = name
    return f


for _n in ("__add__", "__radd__", "__sub__", "__rsub__", "__mul__", "__rmul__", "__truediv__", "__rtruediv__",
           "__neg__", "__eq__", "__ne__", "__lt__", "__le__", "__gt__", "__ge__", "__pow__", "__matmul__"):
    setattr(LazyLogits, _n, _binop(_n))
