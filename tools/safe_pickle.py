"""Read the reference's numpy pickles WITHOUT executing anything from them.

The reference ships `combinatorial_load/{channel_switch_8,setup_8_channels,setup}.p`
(read at /root/reference/xp_load.py:31).  `pickle.load` would execute the
file's GLOBAL/REDUCE opcodes, so instead this walks the opcode stream with
`pickletools.genops` (a pure parser) on a tiny symbolic stack machine:
GLOBAL/REDUCE/BUILD become inert tuples, and the one structural pattern numpy
uses for arrays (`_reconstruct` + `BUILD (1, shape, dtype, fortran, bytes)`) is
turned into an ndarray with `np.frombuffer`.  Nothing is imported or called by
name from the file.  Used only by tools/ in the build container.
"""
import pickletools

import numpy as np


class _Mark:
    pass


_MARK = _Mark()


def _pop_mark(stack):
    items = []
    while True:
        x = stack.pop()
        if x is _MARK:
            break
        items.append(x)
    items.reverse()
    return items


def _materialise(obj):
    """Convert the symbolic objects produced by `load` to plain python/numpy."""
    if isinstance(obj, tuple) and obj and obj[0] == "build":
        _, base, state = obj
        if isinstance(base, tuple) and base[0] == "reduce":
            fn = base[1]
            if fn == ("global", "numpy.core.multiarray", "_reconstruct") or fn == (
                "global", "numpy._core.multiarray", "_reconstruct"):
                _ver, shape, dtype, fortran, raw = state
                dt = _materialise(dtype)
                arr = np.frombuffer(bytes(raw), dtype=dt)
                order = "F" if fortran else "C"
                return arr.reshape(tuple(shape), order=order).copy()
            if fn == ("global", "numpy", "dtype"):
                code = base[2][0]
                endian = state[1]
                if endian in ("|", "="):
                    endian = ""
                return np.dtype(endian + code)
        raise ValueError(f"unsupported BUILD pattern: {base!r}")
    if isinstance(obj, dict):
        return {_materialise(k): _materialise(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_materialise(v) for v in obj]
    if isinstance(obj, tuple) and obj and obj[0] == "reduce" and obj[1] == ("global", "numpy", "dtype"):
        # a memoised dtype referenced again (BINGET) before its BUILD was applied
        return np.dtype("<" + obj[2][0]) if obj[2][0][0] in "fiuc" else np.dtype(obj[2][0])
    if isinstance(obj, tuple) and obj and obj[0] in ("reduce", "global"):
        raise ValueError(f"unsupported object: {obj!r}")
    return obj


def load(path):
    data = open(path, "rb").read()
    stack, memo = [], {}
    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            break
        if name == "MARK":
            stack.append(_MARK)
        elif name == "EMPTY_DICT":
            stack.append({})
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "BININT1", "BININT", "BININT2",
                      "BINFLOAT", "SHORT_BINBYTES", "BINBYTES", "LONG1"):
            stack.append(arg)
        elif name == "NONE":
            stack.append(None)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif name == "TUPLE1":
            stack.append((stack.pop(),))
        elif name == "TUPLE2":
            b = stack.pop(); a = stack.pop(); stack.append((a, b))
        elif name == "TUPLE3":
            c = stack.pop(); b = stack.pop(); a = stack.pop(); stack.append((a, b, c))
        elif name == "TUPLE":
            stack.append(tuple(_pop_mark(stack)))
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name == "STACK_GLOBAL":
            nm = stack.pop(); mod = stack.pop(); stack.append(("global", mod, nm))
        elif name == "REDUCE":
            args = stack.pop(); fn = stack.pop(); stack.append(("reduce", fn, args))
        elif name == "BUILD":
            state = stack.pop(); obj = stack.pop(); stack.append(("build", obj, state))
        elif name == "APPENDS":
            items = _pop_mark(stack); stack[-1].extend(items)
        elif name == "APPEND":
            v = stack.pop(); stack[-1].append(v)
        elif name == "SETITEMS":
            items = _pop_mark(stack)
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif name == "SETITEM":
            v = stack.pop(); k = stack.pop(); stack[-1][k] = v
        else:
            raise ValueError(f"opcode {name} not supported by the safe reader")
    assert len(stack) == 1, stack
    return _materialise(stack[0])
