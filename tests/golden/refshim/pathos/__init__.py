"""pathos stand-in (TEST INFRASTRUCTURE only).

`ProcessPool.map` is sequential but deep-copies each argument first, reproducing
the reference's pickle-to-worker semantics (`aggregator.py:723-724`): the
parent's MPCCalc objects are never mutated by a solve.
"""
import logging


def logger(level=logging.INFO, handler=None, name=None):
    lg = logging.getLogger(name)
    lg.setLevel(level)
    if handler is not None:
        lg.addHandler(handler)
    return lg
