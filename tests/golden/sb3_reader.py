"""No-code reader of the pickled fields in a stable-baselines3 checkpoint's ``data`` file (test infrastructure).

SB3 (2.3.2, ``stable_baselines3/common/save_util.py``) stores the non-JSON attributes of a model -- among them
``_last_obs`` (numpy.ndarray) and ``ep_info_buffer`` (collections.deque of Monitor ``{"r", "l", "t"}`` dicts) -- as
base64 cloudpickle strings.  Unpickling would execute whatever the pickle names, so this reader never calls
``pickle.load``: it walks the opcode stream with ``pickletools.genops`` in a small stack machine that knows only
plain data opcodes, records GLOBAL references as inert names, and interprets the few REDUCE / BUILD shapes that
numpy arrays, dtypes and deques pickle to with its own code (the bytes are handed to ``numpy.frombuffer``; nothing
named in the pickle is imported or called).  Any other callable raises.
"""
import base64
import json
import pickletools
import zipfile

import numpy as np


class Global:
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"Global({self.name})"


class _Mark:
    pass


_MARK = _Mark()


class _DType:
    def __init__(self, code):
        self.code, self.order = code, "|"

    def numpy(self):
        order = self.order if self.order in "<>|=" else "<"
        return np.dtype(self.code).newbyteorder(order) if order != "|" else np.dtype(self.code)


class _Deque(list):
    pass


def _reduce(fn, args):
    """interpret the callables numpy arrays / dtypes and deques pickle to -- with this module's code"""
    if not isinstance(fn, Global):
        raise ValueError(f"REDUCE of a non-global {fn!r}")
    if fn.name == "numpy.dtype":
        return _DType(args[0])
    if fn.name in ("numpy.core.numeric._frombuffer", "numpy._core.numeric._frombuffer"):
        buf, dt, shape, order = args
        a = np.frombuffer(bytes(buf), dtype=dt.numpy()).reshape(shape, order=order)
        return a.copy()
    if fn.name == "collections.deque":
        d = _Deque()
        d.maxlen = args[1] if len(args) > 1 else None
        if args and args[0]:
            d.extend(args[0])
        return d
    raise ValueError(f"refusing to interpret a call of {fn.name}")


def decode(raw):
    """the value a pickle would build, for plain data, numpy arrays (frombuffer protocol), dtypes and deques"""
    stack, memo = [], {}

    def pop_mark():
        items = []
        while True:
            x = stack.pop()
            if x is _MARK:
                return items[::-1]
            items.append(x)

    for op, arg, _pos in pickletools.genops(raw):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        elif n == "STOP":
            break
        elif n == "MARK":
            stack.append(_MARK)
        elif n in ("MEMOIZE",):
            memo[len(memo)] = stack[-1]
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE", "SHORT_BINSTRING", "BINSTRING",
                   "STRING"):
            stack.append(arg)
        elif n in ("BININT", "BININT1", "BININT2", "INT", "LONG1", "LONG4", "LONG", "BINFLOAT", "FLOAT"):
            stack.append(arg)
        elif n in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8", "BYTEARRAY8"):
            stack.append(bytes(arg))
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = stack[-k:]
            del stack[-k:]
            stack.append(tuple(items))
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "LIST":
            stack.append(pop_mark())
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "DICT":
            items = pop_mark()
            stack.append(dict(zip(items[::2], items[1::2])))
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            for k, v in zip(items[::2], items[1::2]):
                stack[-1][k] = v
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            stack.append(Global(f"{mod}.{name}"))
        elif n == "GLOBAL":
            mod, name = arg.split(" ", 1)
            stack.append(Global(f"{mod}.{name}"))
        elif n == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            stack.append(_reduce(fn, args))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, _DType):  # dtype.__setstate__: (version, byteorder, ...)
                obj.order = state[1]
            elif isinstance(obj, _Deque):
                pass
            else:
                raise ValueError(f"BUILD on {type(obj).__name__}")
        else:
            raise ValueError(f"opcode {n} not supported by the no-code reader")
    if len(stack) != 1:
        raise ValueError("malformed pickle")
    return stack[0]


def read_run(zip_path):
    """(JSON-level fields, decoded pickled fields) of an SB3 checkpoint's ``data`` file; decodes only
    _last_obs, _last_episode_starts and ep_info_buffer"""
    with zipfile.ZipFile(zip_path) as z:
        d = json.loads(z.read("data"))
    out = {}
    for k in ("_last_obs", "_last_episode_starts", "ep_info_buffer"):
        v = d.get(k)
        if isinstance(v, dict) and ":serialized:" in v:
            x = decode(base64.b64decode(v[":serialized:"]))
            out[k] = list(x) if isinstance(x, _Deque) else x
    plain = {k: v for k, v in d.items() if not (isinstance(v, dict) and ":serialized:" in v)}
    return plain, out
