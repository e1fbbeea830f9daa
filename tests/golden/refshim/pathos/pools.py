"""pathos.pools stand-in (TEST INFRASTRUCTURE only, tests/golden/make_golden.py).

`ProcessPool.map` forks fresh workers per call, like the reference's per-timestep
pool (`aggregator.py:723-724`): each worker gets a pickled copy of its MPCCalc, so
the parent's objects are never mutated.  Side effects are the redis writes (the
only channel the reference uses) plus golden records; workers return their
journals and the parent replays them in item order, so the result is identical
to a sequential run.
"""
import multiprocessing as mp
import os
import sys
import time

EXTRA = []          # golden records appended by the harness inside a worker
WORKERS = int(os.environ.get("GOLDEN_WORKERS", "8"))
_CALLS, _T0 = [0], time.time()


def _work(args):
    import redis as R
    f, x = args
    R._JOURNAL.clear()
    del EXTRA[:]
    f(x)
    return list(R._JOURNAL), list(EXTRA)


class ProcessPool:
    def __init__(self, nodes=1, **kw):
        self.nodes = nodes

    def map(self, f, items):
        import redis as R
        items = list(items)
        if WORKERS <= 1:
            outs = [_work((f, x)) for x in items]
        else:
            with mp.get_context("fork").Pool(min(WORKERS, max(1, len(items)))) as pool:
                outs = pool.map(_work, [(f, x) for x in items], chunksize=1)
        for journal, extra in outs:
            R.replay(journal)
            EXTRA.extend(extra)
        _CALLS[0] += 1
        print(f"[pool] map #{_CALLS[0]}: {len(items)} items, {time.time() - _T0:.0f}s since start",
              file=sys.stderr, flush=True)
        return [None] * len(items)
