"""toml stand-in over tomli (TEST INFRASTRUCTURE only, tests/golden/make_golden.py)."""
import tomli


def load(f):
    data = f.read()
    if isinstance(data, bytes):
        data = data.decode()
    return tomli.loads(data)


def loads(s):
    return tomli.loads(s)
