"""Stand-in for the absent `numba` package (golden generation only).

The reference decorates `dtw_cpu`/`backtrace` (timing.py:57-105) with
`numba.jit`; JIT compilation does not change their results, so this stand-in
returns the plain Python function.  Used only by oracle/gen_golden.py when it
imports /root/reference in this container; never shipped to the GPU box path.
"""


def jit(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]

    def deco(fn):
        return fn

    return deco


njit = jit
