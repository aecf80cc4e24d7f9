"""ISA encoder/decoder vs the reference encoder's known-answer words.

Fixtures: tests/golden/isa_kat.json (distproc.command_gen outputs on seeded
arguments), tests/golden/cmd_buf_golden.json (the reference's machine-code
golden, python/test/test_outputs/test_linear_compile_globalasm.txt).
"""

import json
import os

import pytest

import distributed_processor_amd.isa as isa


@pytest.fixture(scope='module')
def kat(golden_dir):
    with open(os.path.join(golden_dir, 'isa_kat.json')) as f:
        return json.load(f)


def test_encoder_matches_reference_kat(kat):
    assert len(kat['cases']) > 400
    for case in kat['cases']:
        word = getattr(isa, case['fn'])(*case['args'], **case['kwargs'])
        assert '{:032x}'.format(word) == case['word'], case


def test_twos_complement_kat(kat):
    for case in kat['twos_complement']:
        assert isa.twos_complement(case['value']) == case['tc']
    with pytest.raises(Exception):
        isa.twos_complement(2 ** 31)
    with pytest.raises(Exception):
        isa.twos_complement(-2 ** 31 - 1)


def test_decode_roundtrip(kat):
    for case in kat['cases']:
        w = int(case['word'], 16)
        d = isa.decode(w)
        assert d['op4'] == w >> 124
        if case['fn'] == 'pulse_i':
            f, ph, amp, env, cfg, t = case['args']
            assert (d['freq'], d['phase'], d['amp'], d['env_word'], d['cfg'], d['cmd_time']) == \
                (f, ph, amp, env, cfg, t)
            assert d['freq_we'] and d['phase_we'] and d['amp_we'] and d['env_word_we'] and d['cfg_we']
            assert not (d['freq_sel'] or d['phase_sel'] or d['amp_sel'] or d['env_word_sel'])
        assert isinstance(isa.disasm(w), str)


def test_golden_cmd_buf_decodes(golden_dir):
    with open(os.path.join(golden_dir, 'cmd_buf_golden.json')) as f:
        g = json.load(f)
    core0 = isa.bytes_to_words(bytes.fromhex(g['cores']['0']['cmd_buf']))
    ops = [isa.decode(w)['op'] for w in core0]
    # phase_reset; X90 qdrv @5; read rdrv @21; rdlo @321; done
    assert ops == ['pulse_reset', 'pulse_write_trig', 'pulse_write_trig', 'pulse_write_trig', 'done']
    assert [isa.decode(w)['cmd_time'] for w in core0[1:4]] == [5, 21, 321]
    assert [isa.decode(w)['cfg'] for w in core0[1:4]] == [0, 1, 2]
    u32 = isa.cmd_buf_to_u32(bytes.fromhex(g['cores']['0']['cmd_buf']))
    assert (u32 == isa.words_to_u32(core0)).all()
