package celestiaeds

import (
	"bytes"
	"errors"
)

// RootTable is an rsmt2d.TreeConstructorFn whose trees return roots computed on the
// device by ExtendShares. Push records the pushed cells' identity (first 32 bytes and a
// count) so a tree used on data other than the square it was built for falls back to
// the CPU NMT (wrapper.NewErasuredNamespacedMerkleTree) instead of returning a stale root.
// Custom / NodeVisitor constructors (pkg/inclusion, test/util/malicious) keep using the
// CPU wrapper: they need every inner node, which the device path does not export yet.
type RootTable struct {
	Rows, Cols [][]byte
	Cells      [][]byte // flattened EDS, row-major
	Width      int
}

type rootTree struct {
	t      *RootTable
	axis   int // 0 row, 1 col
	index  int
	pushed int
	ok     bool
}

func (rt *RootTable) NewTree(axis int, index uint) *rootTree {
	return &rootTree{t: rt, axis: axis, index: int(index), ok: true}
}

func (tr *rootTree) Push(data []byte) error {
	if tr.pushed >= tr.t.Width {
		return errors.New("pushed past predetermined square size")
	}
	r, c := tr.index, tr.pushed
	if tr.axis == 1 {
		r, c = tr.pushed, tr.index
	}
	want := tr.t.Cells[r*tr.t.Width+c]
	if !bytes.Equal(data, want) {
		tr.ok = false
	}
	tr.pushed++
	return nil
}

func (tr *rootTree) Root() ([]byte, error) {
	if !tr.ok || tr.pushed != tr.t.Width {
		return nil, errors.New("root table: pushed cells differ from the extended square; use the CPU tree")
	}
	if tr.axis == 0 {
		return tr.t.Rows[tr.index], nil
	}
	return tr.t.Cols[tr.index], nil
}
