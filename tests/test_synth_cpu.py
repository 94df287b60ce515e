"""The parallel per-file generator (bench's C3 proteome) yields exactly the serial generator's
inputs: one RNG stream per genome file, so the worker pool changes nothing."""
import numpy as np

from signature_kmers_amd import synth


def test_parallel_files_equal_serial():
    p = synth.generate_arrays(9000, 100, per_file=2000)
    r, o, l, f, i, funcs = synth.build_inputs(p)
    for workers in (1, 3):
        parts = list(synth.iter_file_inputs(9000, 100, per_file=2000, workers=workers))
        assert len(parts) == 5
        assert np.array_equal(np.concatenate([x[0] for x in parts]), r)
        assert np.array_equal(np.concatenate([x[2] for x in parts]), l)
        assert np.array_equal(np.concatenate([x[3] for x in parts]), f)
        assert np.array_equal(np.concatenate([x[4] for x in parts]), i)
        for x in parts:  # per-file offsets restart at 0
            assert x[1][0] == 0 and np.array_equal(x[1][1:], np.cumsum(x[2][:-1], dtype=np.uint64))
    assert synth.functions(100) == funcs
    # a later shard of files is the same bytes whoever generates it
    tail = list(synth.iter_file_inputs(9000, 100, per_file=2000, first_file=3, n_files=2, workers=2))
    assert np.array_equal(np.concatenate([x[0] for x in tail]), r[int(o[6000]):])
