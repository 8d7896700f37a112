"""pkg/inclusion path computation (host, cel_commitment_paths) against the reference's
own vectors, transcribed from pkg/inclusion/paths_test.go (Test_calculateSubTreeRootCoordinates,
Test_genSubTreeRootPath, Test_calculateCommitPaths)."""
import pytest

L, R = False, True

# (start, end, maxDepth, minDepth) -> [(depth, position)] (paths_test.go:12-319)
COORDS = [
    (0, 4, 3, 1, [(1, 0)]),
    (4, 8, 3, 1, [(1, 1)]),
    (3, 5, 3, 3, [(3, 3), (3, 4)]),
    (3, 4, 3, 3, [(3, 3)]),
    (3, 6, 3, 2, [(3, 3), (2, 2)]),
    (1, 7, 3, 2, [(3, 1), (2, 1), (2, 2), (3, 6)]),
    (1, 7, 3, 3, [(3, 1), (3, 2), (3, 3), (3, 4), (3, 5), (3, 6)]),
    (0, 5, 3, 1, [(1, 0), (3, 4)]),
    (0, 7, 3, 1, [(1, 0), (2, 2), (3, 6)]),
    (0, 8, 3, 0, [(0, 0)]),
    (0, 32, 7, 2, [(2, 0)]),
    (0, 33, 7, 2, [(2, 0), (7, 32)]),
    (0, 31, 7, 3, [(3, 0), (4, 2), (5, 6), (6, 14), (7, 30)]),
    (0, 64, 7, 1, [(1, 0)]),
    (0, 1, 2, 2, [(2, 0)]),
    (0, 19, 6, 3, [(3, 0), (3, 1), (5, 8), (6, 18)]),
]

# (squareSize, start, blobLen) -> {path index: (row, instructions)} (paths_test.go:341-450)
COMMIT = [
    (2, 2, 2, {0: (1, [L]), 1: (1, [R])}),
    (4, 2, 2, {0: (0, [R, L]), 1: (0, [R, R])}),
    (4, 3, 2, {0: (0, [R, R]), 1: (1, [L, L])}),
    (128, 8252, 1, {0: (64, [L, R, R, R, R, L, L])}),
    (128, 0, 8193, {31: (31, [])}),
    (128, 0, 8192, {31: (31, [])}),
    (128, 0, 64, {31: (0, [L, L, R, R, R, R, R])}),
    (128, 0, 65, {31: (0, [L, R, R, R, R, R]), 32: (0, [R, L, L, L, L, L, L])}),
]


@pytest.mark.parametrize("start,end,max_depth,min_depth,expected", COORDS)
def test_subtree_root_coordinates(start, end, max_depth, min_depth, expected):
    from celestia_eds import inclusion
    assert inclusion.calculate_subtree_root_coordinates(max_depth, min_depth, start, end) == expected


def test_gen_subtree_root_path():
    from celestia_eds.inclusion import gen_subtree_root_path as g
    assert g(2, 0) == [L, L] and g(0, 0) == [] and g(3, 0) == [L, L, L]
    assert g(3, 1) == [L, L, R] and g(3, 2) == [L, R, L] and g(5, 16) == [R, L, L, L, L]


@pytest.mark.parametrize("square,start,blob_len,expected", COMMIT)
def test_commitment_paths(square, start, blob_len, expected):
    from celestia_eds import inclusion
    paths = inclusion.calculate_commitment_paths(square, start, blob_len, 64)
    for i, (row, ins) in expected.items():
        assert paths[i] == (row, ins)
    assert len({(r, tuple(p)) for r, p in paths}) == len(paths)  # every path unique


def test_blob_outside_square():
    from celestia_eds import CelError, _lib, inclusion
    with pytest.raises(CelError) as ei:
        inclusion.calculate_commitment_paths(4, 15, 2)
    assert ei.value.status == _lib.ETOOBIG
