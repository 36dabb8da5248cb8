"""Structured JSON-lines logger — the re-provided ``bunyan`` contract.

The reference takes an injectable bunyan logger and derives child loggers per
component (``lib/client.js:34-44``, ``lib/connection-fsm.js:34-36``,
``lib/zk-session.js:51-53``, ``:531-534``).  :class:`Logger` offers the same
``child(**fields)`` / ``trace`` ... ``error`` surface and writes one JSON
object per line (``name``, ``level``, ``time``, ``msg`` plus bound fields).

Level defaults to ``warn`` (quiet library); ``LOG_LEVEL`` or
``ZKMI_LOG_LEVEL`` in the environment override it, like the reference tests'
``LOG_LEVEL`` (``test/basic.test.js:20-23``).
"""

import json
import os
import sys
import time

LEVELS = {'trace': 10, 'debug': 20, 'info': 30, 'warn': 40, 'error': 50,
          'fatal': 60}


def _level_from_env():
    v = os.environ.get('ZKMI_LOG_LEVEL') or os.environ.get('LOG_LEVEL')
    if v and v.lower() in LEVELS:
        return LEVELS[v.lower()]
    return LEVELS['warn']


class Logger(object):

    def __init__(self, name='zkmi', level=None, stream=None, fields=None,
                 _root=None):
        self.name = name
        self._root = _root or self
        if _root is None:
            self.level = _level_from_env() if level is None else (
                LEVELS[level] if isinstance(level, str) else level)
            self.stream = stream or sys.stderr
            self.records = None     # set to a list to capture records
        self.fields = dict(fields or {})

    def child(self, **fields):
        f = dict(self.fields)
        f.update(fields)
        return Logger(self.name, fields=f, _root=self._root)

    def set_level(self, level):
        self._root.level = LEVELS[level] if isinstance(level, str) else level

    def capture(self):
        """Start keeping emitted records in memory (tests)."""
        self._root.records = []
        return self._root.records

    def enabled(self, lvl):
        return LEVELS[lvl] >= self._root.level

    def _log(self, lvl, args):
        root = self._root
        if LEVELS[lvl] < root.level:
            return
        rec = {'name': self.name, 'level': LEVELS[lvl], 'time': time.time()}
        rec.update(self.fields)
        if args and isinstance(args[0], dict):
            rec.update(args[0])
            args = args[1:]
        elif args and isinstance(args[0], BaseException):
            e = args[0]
            rec['err'] = {'name': type(e).__name__, 'message': str(e),
                          'code': getattr(e, 'code', None)}
            args = args[1:]
        if args:
            msg = args[0]
            if len(args) > 1:
                try:
                    msg = msg % tuple(args[1:])
                except (TypeError, ValueError):
                    msg = ' '.join(str(a) for a in args)
            rec['msg'] = str(msg)
        else:
            rec['msg'] = ''
        if root.records is not None:
            root.records.append(rec)
        try:
            root.stream.write(json.dumps(rec, default=str) + '\n')
        except (ValueError, OSError):
            pass

    def trace(self, *a):
        self._log('trace', a)

    def debug(self, *a):
        self._log('debug', a)

    def info(self, *a):
        self._log('info', a)

    def warn(self, *a):
        self._log('warn', a)

    warning = warn

    def error(self, *a):
        self._log('error', a)

    def fatal(self, *a):
        self._log('fatal', a)


def create_logger(name='zkmi', level=None, stream=None, **fields):
    return Logger(name, level=level, stream=stream, fields=fields)
