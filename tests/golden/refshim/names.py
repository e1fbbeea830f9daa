"""`names` stand-in (TEST INFRASTRUCTURE only): deterministic first names."""
_N = [0]


def get_first_name():
    _N[0] += 1
    return f"Home{_N[0]:05d}"
