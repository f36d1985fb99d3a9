from . import train_state  # noqa: F401
from .train_state import TrainState  # noqa: F401
