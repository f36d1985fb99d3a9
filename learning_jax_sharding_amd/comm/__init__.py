from .backend import DistComm, LocalComm, Transfer, get_comm, reset_comm  # noqa: F401
from .collectives import all_gather, all_reduce, all_to_all, exchange, reduce_scatter  # noqa: F401
