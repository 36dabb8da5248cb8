"""Node layer: one ZooKeeper session per rank, RCCL/gloo collectives."""
from .group import SessionGroup, DistributedWatcher, owner_of, \
    METRIC_SCHEMA  # noqa: F401
