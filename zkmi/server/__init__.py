"""In-process fake ZooKeeper (tests / benchmarks)."""
from .fakezk import FakeZKServer, FakeEnsemble, ZKDatabase  # noqa: F401
