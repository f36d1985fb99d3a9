from .api import Jitted, eval_shape, grad, jit, reduce_replica_grads, value_and_grad  # noqa: F401
from .plan import record_plan  # noqa: F401
from .reshard import plan_reshard, reshard  # noqa: F401
