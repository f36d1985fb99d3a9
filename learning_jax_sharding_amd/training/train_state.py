"""``flax.training.train_state.TrainState`` equivalent (``case6_attention.py:171-178,214``)."""
from __future__ import annotations

import dataclasses
from typing import Any, Callable

from ..array import ShardedArray
from ..utils import tree as T

__all__ = ["TrainState"]


@dataclasses.dataclass(eq=False)
class TrainState:
    step: Any
    apply_fn: Callable
    params: Any
    tx: Any
    opt_state: Any

    @classmethod
    def create(cls, *, apply_fn: Callable, params, tx, **kwargs) -> "TrainState":
        opt_state = tx.init(params)
        # the step counter is the optimizer's device-side counter when there is one
        step = opt_state[0].count if hasattr(opt_state[0], "count") else 0
        return cls(step=step, apply_fn=apply_fn, params=params, tx=tx, opt_state=opt_state, **kwargs)

    def apply_gradients(self, *, grads, **kwargs) -> "TrainState":
        if hasattr(self.tx, "apply"):
            new_params, new_opt = self.tx.apply(self.params, grads, self.opt_state)
        else:
            from ..optim.adam import apply_updates
            updates, new_opt = self.tx.update(grads, self.opt_state, self.params)
            new_params = apply_updates(self.params, updates)
        step = new_opt[0].count if hasattr(new_opt[0], "count") else self.step + 1
        return dataclasses.replace(self, step=step, params=new_params, opt_state=new_opt, **kwargs)

    def replace(self, **kwargs) -> "TrainState":
        return dataclasses.replace(self, **kwargs)


def _flatten(s: TrainState):
    return (s.step, s.params, s.opt_state), (s.apply_fn, s.tx)


def _unflatten(aux, ch):
    return TrainState(step=ch[0], apply_fn=aux[0], params=ch[1], tx=aux[1], opt_state=ch[2])


T.register_pytree_node(TrainState, _flatten, _unflatten)
TrainState.__pytree_child_names__ = ("step", "params", "opt_state")
