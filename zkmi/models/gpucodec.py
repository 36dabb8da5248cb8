"""The live connection's control-plane records on the GPU (K9, K11).

With ``ClientConfig.codec_device`` set (e.g. ``'cuda:0'``), a connection
encodes its ConnectRequest with K9 ``encode_connect_requests``, decodes the
server's ConnectResponse with K9 ``decode_connect_responses`` and encodes the
SET_WATCHES frame of a watch resume with K11 ``encode_set_watches`` — the
records of a reconnect, which the reference builds in ``ZKBuffer``
(``lib/zk-buffer.js:22-56``, ``:255-273``) from ``lib/zk-session.js:198-204``
and ``:421-471``.  A SET_WATCHES after a failover carries every watched path
of the session (megabytes for a large watch set), which is where a batched
encoder pays; ConnectRequest / ConnectResponse ride along so the handshake
of a failover never leaves the device codec.

Everything else on the interactive path stays on the host codec
(:mod:`zkmi.codec`): one small record per call is launch-bound on a GPU
(SURVEY §7.4.7).  The bulk API (:mod:`zkmi.models.bulk`) is the batched
data-plane path.
"""

import numpy as np

from ..errors import ZKDecodeError


class GpuControlCodec(object):
    """K9 / K11 for one device; shared by the connections of a client."""

    def __init__(self, device):
        import torch
        from ..ops import batch as B
        self.torch = torch
        self.B = B
        self.device = torch.device(device)
        if self.device.type != 'cuda':
            raise ValueError('codec_device must be a GPU, got %s'
                             % self.device)
        self.calls = {'connect_request': 0, 'connect_response': 0,
                      'set_watches': 0}

    def _host(self, t):
        return bytes(t.cpu().numpy().tobytes())

    def connect_request(self, pkt):
        """Framed ConnectRequest bytes (K9 encode)."""
        with self.torch.cuda.device(self.device):
            out = self.B.encode_connect_requests([pkt], self.device)
            self.calls['connect_request'] += 1
            return self._host(out)

    def connect_response(self, body):
        """Decode one ConnectResponse body (K9 decode) -> packet dict."""
        torch = self.torch
        dev = self.device
        with torch.cuda.device(dev):
            raw = np.frombuffer(bytes(body) or b'\0', np.uint8).copy()
            buf = torch.from_numpy(raw).to(dev)
            ft = self.B.FrameTable(
                torch.zeros(1, dtype=torch.int64, device=dev),
                torch.full((1,), len(body), dtype=torch.int32, device=dev),
                torch.tensor([1, len(body), 0, 0], dtype=torch.int64,
                             device=dev))
            o = self.B.decode_connect_responses(buf, ft, 1)
            vals = torch.stack([o['status'].to(torch.int64),
                                o['protocolVersion'].to(torch.int64),
                                o['timeOut'].to(torch.int64),
                                o['sessionId'], o['passwd_off'],
                                o['passwd_len'].to(torch.int64)])
            st, proto, tmo, sid, po, pl = vals[:, 0].cpu().tolist()
            self.calls['connect_response'] += 1
        if st != 0:
            raise ZKDecodeError('ConnectResponse: truncated record')
        return {'protocolVersion': proto, 'timeOut': tmo, 'sessionId': sid,
                'passwd': bytes(body[po:po + pl])}

    def set_watches(self, pkt):
        """Framed SET_WATCHES bytes (K11 encode) for a packet as
        :func:`zkmi.jute.encode_request` takes it."""
        ev = pkt.get('events') or {}
        with self.torch.cuda.device(self.device):
            out = self.B.encode_set_watches(
                pkt['relZxid'], ev.get('dataChanged', []),
                ev.get('createdOrDestroyed', []),
                ev.get('childrenChanged', []), self.device)
            self.calls['set_watches'] += 1
            return self._host(out)


_CODECS = {}


def for_device(device):
    """The process-wide :class:`GpuControlCodec` of ``device`` (None when
    ``device`` is None)."""
    if device is None:
        return None
    key = str(device)
    c = _CODECS.get(key)
    if c is None:
        c = _CODECS[key] = GpuControlCodec(device)
    return c
