"""In-process fake ZooKeeper server (single node or N-endpoint ensemble) with
fault injection — the test and benchmark backend.

The reference tests spawn real JVM ZooKeepers (``test/zkserver.js``) and
inline misbehaving ``net.createServer`` fakes (``test/nasty.test.js``).  There
is no JVM here, so this module implements the server semantics the client
relies on:

* sessions: create (fresh sid + 16-byte passwd, timeout clamped to
  [2, 20] ticks), resume by sid+passwd, expiry after ``timeout`` without
  traffic (ephemerals deleted, watches fired), CLOSE_SESSION, expired-sid
  reconnect answered with sid 0 and a close;
* tree: ``/`` and ``/zookeeper`` pre-created; NODE_EXISTS / NO_NODE /
  NOT_EMPTY / BAD_VERSION / NO_CHILDREN_FOR_EPHEMERALS; version CAS with -1
  as wildcard; SEQUENTIAL names from the parent's ``cversion`` (10 digits);
  EPHEMERAL owners; stat bookkeeping (czxid/mzxid/pzxid, versions,
  numChildren, dataLength, ms timestamps);
* watches: one-shot per session, ZooKeeper's server tables (data watches
  from getData/exists, child watches from getChildren) and trigger rules,
  including the per-session de-duplication of NodeDeleted;
* SET_WATCHES catch-up against ``relZxid``;
* ensemble: several endpoints share one :class:`ZKDatabase`; stopping an
  endpoint drops its sockets but not its sessions;
* fault hooks: refuse (stopped), accept-and-close, hang, write raw bytes,
  reply protocolVersion=1, pause reads, close/relisten on a schedule.
"""

import os
import time

from .. import consts
from .. import jute
from ..errors import ZKDecodeError
from ..jute import Stat
from ..runtime.loop import new_loop
from ..runtime.tcp import TcpSocket
from ..streams import ZKDecoder


class ZKServerError(Exception):
    def __init__(self, code):
        self.code = code
        super().__init__(code)


class Node(object):
    __slots__ = ('data', 'acl', 'stat', 'children')

    def __init__(self, data, acl, stat):
        self.data = data
        self.acl = acl
        self.stat = stat
        self.children = set()


class SessionRec(object):
    __slots__ = ('sid', 'passwd', 'timeout', 'last_seen', 'ephemerals',
                 'conn', 'closed')

    def __init__(self, sid, passwd, timeout, now):
        self.sid = sid
        self.passwd = passwd
        self.timeout = timeout
        self.last_seen = now
        self.ephemerals = set()
        self.conn = None
        self.closed = False


def _parent(path):
    i = path.rfind('/')
    return '/' if i == 0 else path[:i]


def _valid_path(path):
    if not path or path[0] != '/':
        return False
    if path == '/':
        return True
    if path.endswith('/') or '//' in path or '\0' in path:
        return False
    for comp in path.split('/')[1:]:
        if comp in ('.', '..'):
            return False
    return True


class ZKDatabase(object):
    """The replicated state of the fake ensemble (one per ensemble).

    All methods run on the owning loop thread."""

    def __init__(self, loop, tick_ms=2000, server_id=1):
        self.loop = loop
        self.tick_ms = tick_ms
        self.min_timeout = 2 * tick_ms
        self.max_timeout = 20 * tick_ms
        self.zxid = 0
        self.nodes = {}
        self.sessions = {}
        self.data_watches = {}      # path -> set(sid)
        self.child_watches = {}     # path -> set(sid)
        self._sid_ctr = 0
        self._server_id = server_id
        self.stats = {'requests': 0, 'notifications': 0}
        # path -> every session that ever armed a data watch on it (tests:
        # "only the owner rank holds the ZooKeeper watch")
        self.watch_log = {}
        root = Node(b'', [self._world()], Stat())
        self.nodes['/'] = root
        self._mk('/zookeeper', b'', [self._world()], 0)
        self._expiry_h = None
        self._arm_expiry()

    @staticmethod
    def _world():
        return {'perms': ['READ', 'WRITE', 'CREATE', 'DELETE', 'ADMIN'],
                'id': {'scheme': 'world', 'id': 'anyone'}}

    @staticmethod
    def now_ms():
        return int(time.time() * 1000)

    def _mono(self):
        return self.loop.time_ms()

    # -- sessions -------------------------------------------------------------

    def _arm_expiry(self):
        iv = max(self.tick_ms / 4.0, 5)
        self._expiry_h = self.loop.call_later(iv, self._expiry_tick)

    def _expiry_tick(self):
        now = self._mono()
        for sid, s in list(self.sessions.items()):
            if now - s.last_seen > s.timeout:
                self.expire_session(sid)
        self._arm_expiry()

    def shutdown(self):
        if self._expiry_h is not None:
            self._expiry_h.cancel()
            self._expiry_h = None

    def negotiate_timeout(self, t):
        return int(min(max(t, self.min_timeout), self.max_timeout))

    def new_session(self, timeout):
        self._sid_ctr += 1
        sid = (self._server_id << 56) | \
            ((self.now_ms() & 0xffffffffff) << 16) \
            | (self._sid_ctr & 0xffff)
        passwd = os.urandom(16)
        s = SessionRec(sid, passwd, self.negotiate_timeout(timeout),
                       self._mono())
        self.sessions[sid] = s
        return s

    def touch(self, sid):
        s = self.sessions.get(sid)
        if s is not None:
            s.last_seen = self._mono()

    def expire_session(self, sid):
        s = self.sessions.pop(sid, None)
        if s is None:
            return
        s.closed = True
        self._drop_watches(sid)
        for path in sorted(s.ephemerals, key=len, reverse=True):
            if path in self.nodes:
                try:
                    self.delete(path, -1, None)
                except ZKServerError:
                    pass
        if s.conn is not None:
            s.conn.close_from_server()
            s.conn = None

    close_session = expire_session

    def _drop_watches(self, sid):
        for table in (self.data_watches, self.child_watches):
            for path in list(table):
                table[path].discard(sid)
                if not table[path]:
                    del table[path]

    # -- watches --------------------------------------------------------------

    def _add_watch(self, table, path, sid):
        if sid is None:
            return
        table.setdefault(path, set()).add(sid)
        if table is self.data_watches:
            self.watch_log.setdefault(path, set()).add(sid)

    def _trigger(self, table, path, evtype, suppress=None):
        sids = table.pop(path, None)
        if not sids:
            return set()
        fired = set()
        for sid in sids:
            if suppress is not None and sid in suppress:
                continue
            self._notify(sid, evtype, path)
            fired.add(sid)
        return fired | (suppress or set())

    def _notify(self, sid, evtype, path):
        s = self.sessions.get(sid)
        if s is None or s.conn is None:
            return
        self.stats['notifications'] += 1
        s.conn.send_notification(evtype, path)

    # -- tree -----------------------------------------------------------------

    def _mk(self, path, data, acl, owner):
        self.zxid += 1
        z = self.zxid
        now = self.now_ms()
        st = Stat(z, z, now, now, 0, 0, 0, owner, len(data), 0, z)
        node = Node(data, acl, st)
        self.nodes[path] = node
        if path != '/':
            par = self.nodes[_parent(path)]
            par.children.add(path.rsplit('/', 1)[1])
            par.stat.cversion += 1
            par.stat.numChildren += 1
            par.stat.pzxid = z
        return node

    def create(self, path, data, acl, flags, sid):
        if not _valid_path(path) or path == '/':
            raise ZKServerError('BAD_ARGUMENTS')
        ppath = _parent(path)
        par = self.nodes.get(ppath)
        if par is None:
            raise ZKServerError('NO_NODE')
        if par.stat.ephemeralOwner != 0:
            raise ZKServerError('NO_CHILDREN_FOR_EPHEMERALS')
        mask = jute.flags_to_mask(flags)
        if mask & consts.CREATE_FLAGS['SEQUENTIAL']:
            path = '%s%010d' % (path, par.stat.cversion)
        if path in self.nodes:
            raise ZKServerError('NODE_EXISTS')
        if not acl:
            raise ZKServerError('INVALID_ACL')
        owner = sid if (mask & consts.CREATE_FLAGS['EPHEMERAL']) else 0
        if owner and sid is not None:
            self.sessions[sid].ephemerals.add(path)
        self._mk(path, data, acl, owner or 0)
        self._trigger(self.data_watches, path, 'CREATED')
        self._trigger(self.child_watches, ppath, 'CHILDREN_CHANGED')
        return path

    def delete(self, path, version, sid):
        node = self.nodes.get(path)
        if node is None or path == '/':
            raise ZKServerError('NO_NODE' if node is None else 'BAD_ARGUMENTS')
        if version != -1 and version != node.stat.version:
            raise ZKServerError('BAD_VERSION')
        if node.children:
            raise ZKServerError('NOT_EMPTY')
        self.zxid += 1
        del self.nodes[path]
        owner = node.stat.ephemeralOwner
        if owner:
            s = self.sessions.get(owner)
            if s is not None:
                s.ephemerals.discard(path)
        ppath = _parent(path)
        par = self.nodes[ppath]
        par.children.discard(path.rsplit('/', 1)[1])
        par.stat.cversion += 1
        par.stat.numChildren -= 1
        par.stat.pzxid = self.zxid
        done = self._trigger(self.data_watches, path, 'DELETED')
        self._trigger(self.child_watches, path, 'DELETED', suppress=done)
        self._trigger(self.child_watches, ppath, 'CHILDREN_CHANGED')

    def set_data(self, path, data, version):
        node = self.nodes.get(path)
        if node is None:
            raise ZKServerError('NO_NODE')
        if version != -1 and version != node.stat.version:
            raise ZKServerError('BAD_VERSION')
        self.zxid += 1
        node.data = data
        st = node.stat
        st.version += 1
        st.mzxid = self.zxid
        st.mtime = self.now_ms()
        st.dataLength = len(data)
        self._trigger(self.data_watches, path, 'DATA_CHANGED')
        return st

    def get_data(self, path, watch, sid):
        node = self.nodes.get(path)
        if node is None:
            raise ZKServerError('NO_NODE')
        if watch:
            self._add_watch(self.data_watches, path, sid)
        return node.data, node.stat

    def exists(self, path, watch, sid):
        if watch:
            self._add_watch(self.data_watches, path, sid)
        node = self.nodes.get(path)
        if node is None:
            raise ZKServerError('NO_NODE')
        return node.stat

    def get_children(self, path, watch, sid):
        node = self.nodes.get(path)
        if node is None:
            raise ZKServerError('NO_NODE')
        if watch:
            self._add_watch(self.child_watches, path, sid)
        return sorted(node.children), node.stat

    def get_acl(self, path):
        node = self.nodes.get(path)
        if node is None:
            raise ZKServerError('NO_NODE')
        return node.acl, node.stat

    def set_watches(self, rel, events, sid):
        for path in events.get('dataChanged', []):
            node = self.nodes.get(path)
            if node is None:
                self._notify(sid, 'DELETED', path)
            elif node.stat.mzxid > rel:
                self._notify(sid, 'DATA_CHANGED', path)
            else:
                self._add_watch(self.data_watches, path, sid)
        for path in events.get('createdOrDestroyed', []):
            node = self.nodes.get(path)
            if node is not None:
                self._notify(sid, 'CREATED', path)
            else:
                self._add_watch(self.data_watches, path, sid)
        for path in events.get('childrenChanged', []):
            node = self.nodes.get(path)
            if node is None:
                self._notify(sid, 'DELETED', path)
            elif node.stat.pzxid > rel:
                self._notify(sid, 'CHILDREN_CHANGED', path)
            else:
                self._add_watch(self.child_watches, path, sid)

    # -- request dispatch -----------------------------------------------------

    def handle(self, pkt, sid):
        """Apply one decoded request; returns the reply packet dict."""
        self.stats['requests'] += 1
        op = pkt['opcode']
        rep = {'xid': pkt['xid'], 'opcode': op, 'err': 'OK'}
        try:
            if op == 'GET_DATA':
                rep['data'], rep['stat'] = self.get_data(pkt['path'],
                                                         pkt['watch'], sid)
            elif op == 'EXISTS':
                rep['stat'] = self.exists(pkt['path'], pkt['watch'], sid)
            elif op in ('GET_CHILDREN', 'GET_CHILDREN2'):
                rep['children'], rep['stat'] = self.get_children(
                    pkt['path'], pkt['watch'], sid)
            elif op == 'CREATE':
                rep['path'] = self.create(pkt['path'], pkt['data'],
                                          pkt['acl'], pkt['flags'], sid)
            elif op == 'DELETE':
                self.delete(pkt['path'], pkt['version'], sid)
            elif op == 'SET_DATA':
                rep['stat'] = self.set_data(pkt['path'], pkt['data'],
                                            pkt['version'])
            elif op == 'GET_ACL':
                rep['acl'], rep['stat'] = self.get_acl(pkt['path'])
            elif op == 'SYNC':
                pass
            elif op == 'PING':
                pass
            elif op == 'SET_WATCHES':
                self.set_watches(pkt['relZxid'], pkt['events'], sid)
            else:
                rep['err'] = 'UNIMPLEMENTED'
        except ZKServerError as e:
            rep['err'] = e.code
        rep['zxid'] = self.zxid
        return rep


class _ServerConn(object):
    """One accepted client socket."""

    def __init__(self, server, sock):
        self.server = server
        self.db = server.db
        self.sock = sock
        self.decoder = ZKDecoder()
        self.sid = None
        self.handshook = False
        self.closed = False
        sock.on('data', self._on_data)
        sock.on('end', self._on_end)
        sock.on('close', self._on_close)
        sock.on('error', lambda e: None)

    def _on_end(self):
        self.sock.end()

    def _on_close(self):
        self.closed = True
        self.server.conns.discard(self)
        s = self.db.sessions.get(self.sid) if self.sid is not None else None
        if s is not None and s.conn is self:
            s.conn = None
            # ZooKeeper keeps watches on the connection (ServerCnxn): they
            # die with it and the client re-registers them with SET_WATCHES.
            self.db._drop_watches(s.sid)

    def close_from_server(self):
        if not self.closed:
            self.closed = True
            self.sock.end()
            self.sock.destroy()

    def write(self, body):
        self.sock.write(jute.frame(body))

    def send_notification(self, evtype, path):
        self.write(jute.encode_response({
            'xid': consts.XID_NOTIFICATION, 'zxid': -1, 'err': 'OK',
            'opcode': 'NOTIFICATION', 'type': evtype,
            'state': 'SYNC_CONNECTED', 'path': path}))

    def _on_data(self, chunk):
        srv = self.server
        if srv.paused:
            srv.held.append((self, chunk))
            return
        bodies, err = self.decoder.feed(chunk)
        for body in bodies:
            if self.closed:
                return
            if not self.handshook:
                self._handshake(body)
            else:
                self._request(body)
        if err is not None:
            self.close_from_server()

    def _handshake(self, body):
        try:
            req = jute.decode_connect_request(body)
        except ZKDecodeError:
            self.close_from_server()
            return
        db = self.db
        srv = self.server
        self.handshook = True
        if srv.reply_version is not None:
            self.write(jute.encode_connect_response({
                'protocolVersion': srv.reply_version,
                'timeOut': req['timeOut'], 'sessionId': 0x1234,
                'passwd': os.urandom(16)}, read_only=False))
            return
        sid = req['sessionId']
        if sid == 0:
            s = db.new_session(req['timeOut'])
        else:
            s = db.sessions.get(sid)
            if s is None or s.passwd != req['passwd']:
                self.write(jute.encode_connect_response({
                    'protocolVersion': 0, 'timeOut': 0, 'sessionId': 0,
                    'passwd': b'\0' * 16}, read_only=False))
                self.sock.end()
                self.server.loop.call_later(50, self.close_from_server)
                return
            # A session moving to this connection drops its old one.
            if s.conn is not None and s.conn is not self:
                s.conn.close_from_server()
            self.db._drop_watches(s.sid)
            s.last_seen = db._mono()
        s.conn = self
        self.sid = s.sid
        self.write(jute.encode_connect_response({
            'protocolVersion': 0, 'timeOut': s.timeout, 'sessionId': s.sid,
            'passwd': s.passwd}, read_only=False))

    def _request(self, body):
        db = self.db
        s = db.sessions.get(self.sid)
        if s is None or s.conn is not self:
            self.close_from_server()
            return
        s.last_seen = db._mono()
        try:
            pkt = jute.decode_request(body)
        except (ZKDecodeError, ValueError, UnicodeDecodeError):
            self.close_from_server()
            return
        if pkt['opcode'] == 'CLOSE_SESSION':
            self.write(jute.encode_response({
                'xid': pkt['xid'], 'zxid': db.zxid, 'err': 'OK',
                'opcode': 'CLOSE_SESSION'}))
            s.conn = None
            db.close_session(self.sid)
            self.sock.end()
            self.server.loop.call_later(20, self.close_from_server)
            return
        rep = db.handle(pkt, self.sid)
        self.write(jute.encode_response(rep))


class FakeZKServer(object):
    """One listening endpoint.  ``FakeZKServer(port=0)`` picks a free port;
    ``servers()`` gives the client ``servers=`` list."""

    def __init__(self, db=None, host='127.0.0.1', port=0, loop=None,
                 tick_ms=2000, server_id=1):
        self.loop = loop or new_loop(name='fakezk')
        self._own_loop = loop is None
        self.db = db or self.loop.run(lambda: ZKDatabase(self.loop, tick_ms,
                                                         server_id))
        self.host = host
        self.port = port
        self.conns = set()
        self.paused = False
        self.held = []
        self.mode = 'normal'
        self.raw_writes = []        # [(delay_ms, bytes)] for mode 'write'
        self.reply_version = None
        self.accepted = 0
        self._srv = None
        self.start()

    # -- lifecycle ------------------------------------------------------------

    def start(self):
        factory = TcpSocket.protocol_for(self.loop, self._on_accept)
        self._srv = self.loop.start_server(factory, self.host, self.port)
        self.port = self._srv.port
        return self

    def stop(self, kill_sessions=False):
        """Stop listening and drop every connection (a killed server)."""
        def go():
            if self._srv is not None:
                self._srv.close()
                self._srv = None
            for c in list(self.conns):
                c.close_from_server()
            self.conns.clear()
            if kill_sessions:
                for sid in list(self.db.sessions):
                    self.db.expire_session(sid)
        self.loop.run(go)

    def shutdown(self):
        self.stop()
        if self._own_loop:
            self.loop.run(self.db.shutdown)
            self.loop.stop()

    def run(self, fn):
        return self.loop.run(fn)

    @property
    def address(self):
        return {'address': self.host, 'port': self.port}

    def servers(self):
        return [self.address]

    # -- faults ---------------------------------------------------------------

    def set_mode(self, mode, raw_writes=None, reply_version=None):
        """``normal`` | ``close`` (accept then close) | ``hang`` | ``write``
        (send ``raw_writes`` = [(delay_ms, bytes)] then idle) |
        ``bad_version`` (reply protocolVersion=1)."""
        self.mode = mode
        self.raw_writes = list(raw_writes or [])
        self.reply_version = 1 if mode == 'bad_version' else reply_version

    def pause_reads(self):
        self.paused = True

    def resume_reads(self):
        def go():
            self.paused = False
            held, self.held = self.held, []
            for c, chunk in held:
                c._on_data(chunk)
        self.loop.run(go)

    def drop_connections(self):
        self.loop.run(lambda: [c.close_from_server()
                               for c in list(self.conns)])

    def _on_accept(self, sock):
        self.accepted += 1
        if self.mode == 'close':
            sock.destroy()
            return
        if self.mode == 'hang':
            sock.on('error', lambda e: None)
            self.conns.add(_Hung(sock))
            return
        if self.mode == 'write':
            sock.on('error', lambda e: None)
            self.conns.add(_Hung(sock))
            for delay, data in self.raw_writes:
                if delay:
                    self.loop.call_later(delay, sock.write, data)
                else:
                    sock.write(data)
            return
        c = _ServerConn(self, sock)
        self.conns.add(c)

    # -- out-of-band mutations (the reference tests' zk.cli(...)) -------------

    def cli_create(self, path, data=b'', ephemeral_sid=None, flags=()):
        return self.run(lambda: self.db.create(
            path, data, [ZKDatabase._world()], list(flags), ephemeral_sid))

    def cli_set(self, path, data, version=-1):
        return self.run(lambda: self.db.set_data(path, data, version))

    def cli_get(self, path):
        def go():
            n = self.db.nodes.get(path)
            return None if n is None else n.data
        return self.run(go)

    def cli_delete(self, path, version=-1):
        return self.run(lambda: self.db.delete(path, version, None))

    def cli_exists(self, path):
        return self.run(lambda: path in self.db.nodes)


class _Hung(object):
    def __init__(self, sock):
        self.sock = sock

    def close_from_server(self):
        self.sock.destroy()


class FakeEnsemble(object):
    """``n`` endpoints sharing one database (the 3-node ensemble of
    ``test/multi-node.test.js``)."""

    def __init__(self, n=3, tick_ms=2000):
        self.loop = new_loop(name='fakezk-ens')
        self.db = self.loop.run(lambda: ZKDatabase(self.loop, tick_ms, 1))
        self.members = [FakeZKServer(db=self.db, loop=self.loop,
                                     server_id=i + 1) for i in range(n)]

    def __getitem__(self, i):
        return self.members[i]

    def servers(self):
        return [m.address for m in self.members]

    def index_of(self, port):
        for i, m in enumerate(self.members):
            if m.port == port:
                return i
        return -1

    def outage(self, i, sets=()):
        """Kill member ``i`` (its sockets close, its sessions stay alive, as
        a killed ZooKeeper server, test/multi-node.test.js:309-316) and apply
        ``sets`` = [(path, data)] in the same loop turn, so every write lands
        while the member's clients are detached: their reconnect must replay
        the changes through SET_WATCHES (zk-session.js:421-471).  Returns
        the zxid after the writes."""
        def go():
            self.members[i].stop()
            for p, d in sets:
                self.db.set_data(p, d, -1)
            return self.db.zxid
        return self.loop.run(go)

    def shutdown(self):
        for m in self.members:
            m.stop()
        self.loop.run(self.db.shutdown)
        self.loop.stop()
