"""Tunables the reference hard-codes, exposed with the reference's defaults
(SURVEY §5 "Config / flags").  Tests shrink the time constants so that
expiry / ping-timeout scenarios run in seconds."""

from dataclasses import dataclass, field
from typing import Optional


@dataclass
class RecoveryPolicy(object):
    timeout: int = 5000      # ms allowed for one attempt
    retries: int = 3         # attempts before a backend counts as failed
    delay: int = 1000        # initial backoff, doubled per failure
    max_delay: int = 30000   # backoff cap (monitor mode)


@dataclass
class ClientConfig(object):
    # lib/connection-fsm.js:201-203 — ping every max(T/4, floor)
    ping_interval_divisor: float = 4.0
    ping_floor_ms: int = 2000
    # lib/connection-fsm.js:439-441 — ping timeout max(T/8, floor)
    ping_timeout_divisor: float = 8.0
    ping_timeout_floor_ms: int = 2000
    # lib/zk-streams.js:23
    max_packet: int = 16 * 1024 * 1024
    # lib/zk-session.js:35-36 — watcher double-check 4h + U(0, 8h)
    doublecheck_ms: int = 4 * 3600 * 1000
    doublecheck_rand_ms: int = 8 * 3600 * 1000
    # lib/client.js:93-114 — cueball ConnectionSet options
    connect_policy: RecoveryPolicy = field(
        default_factory=lambda: RecoveryPolicy(3000, 3, 500))
    default_policy: RecoveryPolicy = field(
        default_factory=lambda: RecoveryPolicy(5000, 3, 1000))
    target: int = 1
    maximum: int = 3
    decoherence_interval_s: float = 600.0
    shuffle_backends: bool = False
    # lib/client.js:173-176 — closing progress log interval
    close_log_interval_ms: int = 5000
    # not in the reference: a GPU (e.g. 'cuda:0') whose HIP kernels encode
    # the ConnectRequest (K9) and SET_WATCHES (K11) records and decode the
    # ConnectResponse (K9) of every (re)connect (models/gpucodec.py)
    codec_device: Optional[str] = None
    # not in the reference: the native completion path (README).  Replies
    # to outstanding requests settled in the native loop's read path
    # (Transport.route); requests made off the loop thread encoded and sent
    # from the calling thread (ZKConnectionFSM.request_direct); and how long
    # call_sync polls for the reply before it sleeps (None: 100 us on hosts
    # with >= 16 CPUs, else 0)
    native_route: bool = True
    # the session's watch events in the native engine (csrc/host/
    # zk_watch.cpp) instead of one Python state machine per (path, event)
    native_watch: bool = True
    direct_send: bool = True
    sync_spin_us: Optional[float] = None
