"""``optax`` equivalent."""
from .adam import (  # noqa: F401
    EmptyState, GradientTransformation, ScaleByAdamState, adam, adamw, apply_updates, chain, scale, sgd,
)
