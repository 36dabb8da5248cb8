"""zkmi — a ZooKeeper client framework built for AMD MI355X.

Public surface (parity with node-zkstream ``lib/index.js:56-61``): ``Client``
and the error classes.  See README.md for the layer map.
"""

from .errors import (ZKError, ZKProtocolError, ZKPingTimeoutError,  # noqa
                     ZKNotConnectedError)
from .models.client import Client  # noqa: F401
from .config import ClientConfig, RecoveryPolicy  # noqa: F401
from .jute import Stat  # noqa: F401
from . import consts  # noqa: F401

__version__ = '0.1.0'
