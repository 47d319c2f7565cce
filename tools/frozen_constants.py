"""Read the constant tensors of a frozen TorchScript deployment WITHOUT
unpickling or executing anything from it (build container only).

``constants.pkl`` is walked with ``pickletools.genops`` (a parser) by a tiny
stack machine that understands only the opcodes a list of
``torch._utils._rebuild_tensor_v2(storage, offset, shape, stride, ...)``
records uses; no global is imported, nothing is called.  The tensor bytes are
the raw little-endian storages ``<archive>/constants/<key>``.  Returns the
constants in order (the frozen code's CONSTANTS.c0, c1, ...).
"""
import pickletools
import zipfile

import numpy as np

_DTYPES = {'FloatStorage': '<f4', 'DoubleStorage': '<f8', 'LongStorage': '<i8',
           'IntStorage': '<i4', 'BoolStorage': '?'}


class _Global:
    def __init__(self, name):
        self.name = name


def _parse(data):
    stack, memo, marks = [], {}, []
    for op, arg, _ in pickletools.genops(data):
        n = op.name
        if n in ('PROTO', 'FRAME', 'STOP'):
            continue
        if n == 'MARK':
            marks.append(len(stack))
        elif n == 'GLOBAL':
            stack.append(_Global(arg.replace(' ', '.')))
        elif n in ('BINPUT', 'LONG_BINPUT', 'MEMOIZE'):
            memo[arg if n != 'MEMOIZE' else len(memo)] = stack[-1]
        elif n in ('BINGET', 'LONG_BINGET'):
            stack.append(memo[arg])
        elif n in ('BINUNICODE', 'SHORT_BINUNICODE', 'BININT1', 'BININT2', 'BININT',
                   'BINFLOAT', 'LONG1'):
            stack.append(arg)
        elif n == 'NEWFALSE':
            stack.append(False)
        elif n == 'NEWTRUE':
            stack.append(True)
        elif n == 'NONE':
            stack.append(None)
        elif n == 'EMPTY_TUPLE':
            stack.append(())
        elif n == 'TUPLE':
            k = marks.pop()
            t = tuple(stack[k:])
            del stack[k:]
            stack.append(t)
        elif n in ('TUPLE1', 'TUPLE2', 'TUPLE3'):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == 'BINPERSID':
            pid = stack.pop()   # ('storage', storage_type, key, location, numel)
            stack.append({'storage': pid[1].name.rsplit('.', 1)[-1], 'key': pid[2],
                          'numel': pid[4]})
        elif n == 'REDUCE':
            args = stack.pop()
            fn = stack.pop()
            if fn.name.endswith('_rebuild_tensor_v2'):
                st, off, shape, stride = args[0], args[1], args[2], args[3]
                stack.append({**st, 'offset': off, 'shape': tuple(shape), 'stride': tuple(stride)})
            elif fn.name.endswith('OrderedDict'):
                stack.append({})
            else:
                raise ValueError(f'unexpected callable {fn.name}')
        else:
            raise ValueError(f'unexpected pickle opcode {n}')
    assert len(stack) == 1
    return stack[0]


def frozen_constants(archive):
    z = zipfile.ZipFile(archive)
    root = z.namelist()[0].split('/')[0]
    recs = _parse(z.read(f'{root}/constants.pkl'))
    out = []
    for r in recs:
        dt = np.dtype(_DTYPES[r['storage']])
        raw = np.frombuffer(z.read(f'{root}/constants/{r["key"]}'), dtype=dt)
        a = np.lib.stride_tricks.as_strided(raw[r['offset']:], shape=r['shape'],
                                            strides=tuple(dt.itemsize * s for s in r['stride']))
        out.append(np.array(a))
    return out
