"""Refusal of malformed libwavernn .bin files (host code, no device).

The .bin reader (csrc/binfile.cpp, the C-ABI's wrnn_bin_read) parses files a user hands it, in
a format whose reference reader has a known index bug: ``colIdx`` is ``int8_t``
(vocoder/libwavernn/*/src/wavernn.h:28), so column-group indices past 127 -- every matrix wider
than 508 columns, e.g. fatchord's 544-wide rnn2 / fc1 / fc2 -- wrap negative there. Here the
index stream is read as uint8 (convert.py:60-74 writes ``np.uint8``) and every index is bounds
checked. Each malformed file must come back as ValueError ("libwavernn .bin: ..."), never a
crash; tests/test_sanitizers.py runs this file against the ASan + UBSan build of the reader.
"""
import io
import struct

import numpy as np
import pytest

MT = 'geneing-wavernn'  # smallest topology: 1 GRU, 2 linears


def _hp():
    from wavernn_amd.base import hparams_for
    return hparams_for(MT).copy(bits=9, mode='BITS')


def _file(sd=None, el_size=4):
    from wavernn_amd import convert
    from wavernn_amd.synth import synth_state_dict
    hp = _hp()
    sd = sd if sd is not None else synth_state_dict(hp, MT, seed=5)
    f = io.BytesIO()
    convert.write_bin(f, sd, hp, MT, el_size=el_size)
    return f.getvalue(), sd


def _read(data, hp=None, mt=MT):
    from wavernn_amd import convert
    return convert.read_bin(data, hp or _hp(), mt)


def _layer_offsets(data):
    """Byte offset of every layer header (type int32 + 64-byte name) of a geneing file, by
    walking the records the way the reader does."""
    hp = _hp()
    off = 16
    out = []

    def i32(o):
        return struct.unpack_from('@i', data, o)[0]

    def comp(o):
        nw = i32(o)
        o += 4 + 4 * nw
        ni = i32(o)
        return o + 4 + ni
    while off < len(data):
        t = i32(off)
        out.append((t, off))
        o = off + 68
        if t == 1:    # Conv1d
            es, hb, ci, co, k = struct.unpack_from('@5i', data, o)
            o += 20 + 4 * co * ci * k + (4 * co if hb else 0)
        elif t == 2:  # Conv2d
            es, k = struct.unpack_from('@2i', data, o)
            o += 8 + 4 * k
        elif t == 3:  # BatchNorm
            es, n = struct.unpack_from('@2i', data, o)
            o += 12 + 16 * n
        elif t == 4:  # Linear
            es, rows, cols = struct.unpack_from('@3i', data, o)
            o = comp(o + 12) + 4 * rows
        elif t == 5:  # GRU
            es, hid, inp = struct.unpack_from('@3i', data, o)
            o += 12
            for _ in range(6):
                o = comp(o)
            o += 6 * 4 * hid
        elif t == 6:  # Stretch2d
            o += 8
        else:
            raise AssertionError(t)
        off = o
    assert off == len(data)
    return out


def test_walker_matches_reader():
    data, sd = _file()
    back = _read(data)
    assert set(back) >= {'I.weight', 'rnn1.weight_ih_l0', 'fc3.weight'}
    kinds = [t for t, _ in _layer_offsets(data)]
    assert kinds.count(5) == 1 and kinds.count(4) == 3  # rnn1; I, fc1, fc3


@pytest.mark.parametrize('cut', [1, 3, 15, 16, 17, 83, 84, 1000, 0.25, 0.5, 0.75, -1, -4, -5])
def test_truncated_file(cut):
    data, _ = _file()
    n = int(len(data) * cut) if isinstance(cut, float) else (cut if cut > 0 else len(data) + cut)
    with pytest.raises(ValueError, match='Cannot open file|libwavernn .bin'):
        _read(data[:n])


def _linear_record(data, which):
    """(offset of the index-count int32, nw, ni, rows, cols) of the which-th Linear layer."""
    off = [o for t, o in _layer_offsets(data) if t == 4][which]
    es, rows, cols = struct.unpack_from('@3i', data, off + 68)
    nw_off = off + 68 + 12
    nw = struct.unpack_from('@i', data, nw_off)[0]
    ni_off = nw_off + 4 + 4 * nw
    ni = struct.unpack_from('@i', data, ni_off)[0]
    return nw_off, ni_off, nw, ni, rows, cols


@pytest.mark.parametrize('value', [2 ** 31 - 1, 2 ** 30, -1, -2 ** 31])
def test_array_length_beyond_the_file(value):
    """A weight count / index count larger than the file, or negative."""
    data, _ = _file()
    nw_off, ni_off, nw, ni, rows, cols = _linear_record(data, 1)
    for at in (nw_off, ni_off):
        bad = bytearray(data)
        bad[at:at + 4] = struct.pack('@i', value)
        with pytest.raises(ValueError, match='libwavernn .bin'):
            _read(bytes(bad))


def test_header_counts_beyond_the_file():
    """A layer header whose declared sizes do not match the model is refused before any array
    is read (Conv1d out channels, BatchNorm width, GRU hidden size)."""
    data, _ = _file()
    offs = _layer_offsets(data)
    for kind, field in ((1, 12), (3, 4), (5, 4)):
        off = [o for t, o in offs if t == kind][0]
        bad = bytearray(data)
        bad[off + 68 + field:off + 72 + field] = struct.pack('@i', 1 << 28)
        with pytest.raises(ValueError, match='does not match'):
            _read(bytes(bad))


@pytest.mark.parametrize('group', [128, 200, 254])
def test_column_group_index_out_of_range(group):
    """fc1 is 192 columns wide (48 groups): an index the reference's int8 colIdx would read as
    negative (>= 128), or past the row, is refused."""
    data, _ = _file()
    nw_off, ni_off, nw, ni, rows, cols = _linear_record(data, 1)  # fc1
    assert cols // 4 < group
    bad = bytearray(data)
    bad[ni_off + 4] = group  # first index of row 0
    with pytest.raises(ValueError, match='bad group index'):
        _read(bytes(bad))


def test_unordered_group_indices():
    data, _ = _file()
    nw_off, ni_off, nw, ni, rows, cols = _linear_record(data, 1)
    bad = bytearray(data)
    bad[ni_off + 4], bad[ni_off + 5] = bad[ni_off + 5], bad[ni_off + 4]  # 0, 1 -> 1, 0
    with pytest.raises(ValueError, match='bad group index'):
        _read(bytes(bad))


def test_index_stream_shorter_than_the_matrix():
    data, _ = _file()
    nw_off, ni_off, nw, ni, rows, cols = _linear_record(data, 1)
    bad = bytearray(data)
    bad[ni_off + 4:ni_off + 4 + ni] = b'\xff' * ni  # every row empty: weights left over
    with pytest.raises(ValueError, match='do not match'):
        _read(bytes(bad))


def test_zero_row_layer():
    """A Linear record declaring 0 rows (or 0 columns) does not match any model."""
    data, _ = _file()
    off = [o for t, o in _layer_offsets(data) if t == 4][2]  # fc3
    for field in (4, 8):
        bad = bytearray(data)
        bad[off + 68 + field:off + 72 + field] = struct.pack('@i', 0)
        with pytest.raises(ValueError, match='does not match'):
            _read(bytes(bad))


def test_wrong_layer_type():
    data, _ = _file()
    off = [o for t, o in _layer_offsets(data) if t == 5][0]
    bad = bytearray(data)
    bad[off:off + 4] = struct.pack('@i', 99)
    with pytest.raises(ValueError, match='expected a GRU layer'):
        _read(bytes(bad))


def test_invalid_configuration_is_refused():
    """The topology struct comes from the caller: out-of-range fields are refused, not used."""
    import ctypes
    from wavernn_amd import _abi
    from wavernn_amd.convert import config_for
    data, _ = _file()
    lib = _abi.load_library()
    cb = _abi.TENSOR_FN(lambda *a: 0)
    for field, value in (('n_upsample', 9), ('n_upsample', 0), ('bits', 40), ('res_blocks', -1),
                         ('rnn_dims', 0)):
        cfg = config_for(_hp(), MT)
        cfg.mode = _abi.WRNN_MODE_RAW
        setattr(cfg, field, value)
        assert lib.wrnn_bin_read(data, len(data), ctypes.byref(cfg), cb, None) == _abi.WRNN_ERR_INVALID
        assert 'invalid model configuration' in _abi.last_error()


def test_wide_matrix_groups_past_127_land_in_place():
    """fatchord's rnn2 input is 544 wide (136 groups): groups 128..135 (negative in the
    reference's int8 colIdx) must land at columns 512..543."""
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    from wavernn_amd.synth import synth_state_dict
    mt = 'fatchord-wavernn'
    hp = hparams_for(mt).copy(bits=9)
    sd = {k: np.array(v, np.float32) for k, v in synth_state_dict(hp, mt, seed=2).items()}
    W = sd['rnn2.weight_ih_l0']
    assert W.shape[1] == 544
    W[:, :512] = 0  # only the groups past 127 survive the compression
    f = io.BytesIO()
    convert.write_bin(f, sd, hp, mt)
    back = convert.read_bin(f.getvalue(), hp, mt)['rnn2.weight_ih_l0']
    assert np.array_equal(back, W) and np.abs(back[:, 512:]).sum() > 0


def test_random_mutations_never_crash():
    """200 seeded single-word corruptions of a valid file: each is read or refused cleanly."""
    data, _ = _file()
    rng = np.random.default_rng(0)
    refused = 0
    for _ in range(200):
        bad = bytearray(data)
        at = int(rng.integers(0, len(data) // 4)) * 4
        bad[at:at + 4] = struct.pack('@i', int(rng.choice([0, -1, 255, 1 << 20, int(rng.integers(-2 ** 31, 2 ** 31))])))
        try:
            _read(bytes(bad))
        except ValueError as e:
            assert 'libwavernn .bin' in str(e) or 'Cannot open file' in str(e)
            refused += 1
    assert refused > 0


def test_fp16_writer_refuses_out_of_range_values():
    """a finite weight past the fp16 range would be written as inf; refused, naming
    the tensor."""
    from wavernn_amd.synth import synth_state_dict
    sd = {k: np.array(v, np.float32) for k, v in synth_state_dict(_hp(), MT, seed=5).items()}
    sd['upsample.resnet.batch_norm.running_var'][3] = 1e5
    with pytest.raises(ValueError, match='batch_norm.running_var.*fp16 range'):
        _file(sd, el_size=2)
    _file(sd, el_size=4)  # fine in fp32
