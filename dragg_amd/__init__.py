"""dragg_amd: MI355X-native batched home-MPC solver for DRAGG (corymosiman12/dragg).

The hot path -- every home's HEMS MPC solve of a timestep (`dragg/mpc_calc.py`) -- runs as
ONE gfx950 HIP launch through the C ABI in include/dragg_mi355x.h (libdragg_mi355x.so).
"""
__version__ = "0.1.0"
