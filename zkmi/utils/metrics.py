"""Counter registry — the re-provided ``artedi`` contract.

The reference registers ``zookeeper_events{evtype}`` (``lib/client.js:29``,
``:58-61``, ``:222-235``) and ``zookeeper_notifications{event}``
(``lib/zk-session.js:25``, ``:62-65``, ``:413-415``) on an injectable
collector.  Same names and labels here; :meth:`Collector.collect` renders
Prometheus text, and :meth:`Collector.as_vector` flattens the counters for
the node-level RCCL all-reduce (R4, :mod:`zkmi.parallel`).
"""

import threading


class Counter(object):

    def __init__(self, name, help=''):
        self.name = name
        self.help = help
        self.values = {}
        self._lock = threading.Lock()

    def increment(self, labels=None, value=1):
        key = tuple(sorted((labels or {}).items()))
        with self._lock:
            self.values[key] = self.values.get(key, 0) + value

    add = increment

    def get(self, labels=None):
        key = tuple(sorted((labels or {}).items()))
        return self.values.get(key, 0)


class Collector(object):

    def __init__(self):
        self.counters = {}

    def counter(self, name, help=''):
        c = self.counters.get(name)
        if c is None:
            c = Counter(name, help)
            self.counters[name] = c
        return c

    def getCollector(self, name):
        return self.counters[name]

    get_collector = getCollector

    def collect(self):
        lines = []
        for name in sorted(self.counters):
            c = self.counters[name]
            lines.append('# HELP %s %s' % (name, c.help))
            lines.append('# TYPE %s counter' % name)
            for key in sorted(c.values):
                lab = ','.join('%s="%s"' % kv for kv in key)
                lines.append('%s{%s} %d' % (name, lab, c.values[key]) if lab
                             else '%s %d' % (name, c.values[key]))
        return '\n'.join(lines) + '\n'

    def as_vector(self, schema):
        """Values for ``schema`` = [(name, labels_dict), ...] in order."""
        out = []
        for name, labels in schema:
            c = self.counters.get(name)
            out.append(c.get(labels) if c is not None else 0)
        return out


def create_collector():
    return Collector()


METRIC_ZK_EVENT_COUNTER = 'zookeeper_events'
METRIC_ZK_NOTIFICATION_COUNTER = 'zookeeper_notifications'
