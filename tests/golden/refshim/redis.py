"""In-memory redis stand-in for tests/golden/make_golden.py (TEST INFRASTRUCTURE only).

Mirrors the redis-py behaviour the reference relies on (`dragg/redis_client.py:16`,
`decode_responses=True`): every value comes back as ``str``.  Floats are encoded
with ``repr(float(x))`` (the numpy-1.x era repr the reference was written against),
ints with ``str``.  One process-wide store, like one redis server.
"""
_STORE = {}
_JOURNAL = []   # writes made in this process since the last clear (see pathos stand-in)


class DataError(Exception):
    pass


def _enc(v):
    if isinstance(v, bool):
        raise DataError("bool")
    if isinstance(v, str):
        return v
    if isinstance(v, bytes):
        return v.decode()
    try:
        import numpy as np
        if isinstance(v, np.integer):
            return str(int(v))
        if isinstance(v, np.floating):
            return repr(float(v))
    except ImportError:
        pass
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return repr(v)
    raise DataError(f"Invalid input of type: {type(v).__name__}")


class ConnectionPool:
    def __init__(self, **kw):
        self.kw = kw


class Redis:
    def __init__(self, connection_pool=None, **kw):
        self.s = _STORE

    def __deepcopy__(self, memo):  # a pickled client still talks to the same server
        return self

    def __reduce__(self):
        return (Redis, ())

    def flushall(self):
        self.s.clear()

    def set(self, k, v):
        self.s[k] = _enc(v)

    def get(self, k):
        return self.s.get(k)

    def delete(self, *ks):
        for k in ks:
            self.s.pop(k, None)

    def rpush(self, k, *vals):
        self.s.setdefault(k, []).extend(_enc(v) for v in vals)

    def lrange(self, k, a, b):
        lst = self.s.get(k, [])
        b = len(lst) - 1 if b == -1 else b
        return list(lst[a:b + 1])

    def hset(self, k, f, v):
        self.s.setdefault(k, {})[f] = _enc(v)
        _JOURNAL.append((k, f, self.s[k][f]))

    def hgetall(self, k):
        return dict(self.s.get(k, {}))


StrictRedis = Redis


def replay(journal):
    for k, f, v in journal:
        _STORE.setdefault(k, {})[f] = v
