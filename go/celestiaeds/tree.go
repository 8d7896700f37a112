package celestiaeds

import (
	"bytes"
	"fmt"

	"github.com/celestiaorg/celestia-app/v3/pkg/appconsts"
	"github.com/celestiaorg/celestia-app/v3/pkg/wrapper"
	"github.com/celestiaorg/rsmt2d"
)

// RootTable serves rsmt2d trees whose roots the device already computed in
// ExtendShares. Its NewTree method is an rsmt2d.TreeConstructorFn
// (func(rsmt2d.Axis, uint) rsmt2d.Tree), the type wrapper.NewConstructor returns
// (/root/reference/pkg/wrapper/nmt_wrapper.go:14-17,73-86), so it can be handed to
// rsmt2d.ImportExtendedDataSquare in place of the wrapper constructor.
//
// A tree answers from the table only while every pushed cell is byte-identical to the
// cell the device hashed. On the first difference it replays the cells pushed so far
// into the reference tree (wrapper.NewErasuredNamespacedMerkleTree) and delegates every
// later Push and the Root to it, so a tree used on other data returns the reference's
// root and the reference's Push errors. Custom / NodeVisitor constructors
// (pkg/inclusion/nmt_caching.go:96-104, test/util/malicious/tree.go:36-71) are not
// wrapped: callers that pass them keep using them.
type RootTable struct {
	Rows, Cols [][]byte // 2k roots each (90 B), as cel_extend_shares returned them
	Cells      [][]byte // the flattened 2k x 2k square the roots were computed over
	Width      int      // 2k
}

var (
	_ rsmt2d.TreeConstructorFn = (&RootTable{}).NewTree
	_ rsmt2d.Tree              = &rootTree{}
)

// NewTree is the rsmt2d.TreeConstructorFn.
func (rt *RootTable) NewTree(axis rsmt2d.Axis, index uint) rsmt2d.Tree {
	return &rootTree{t: rt, axis: axis, index: index}
}

type rootTree struct {
	t      *RootTable
	axis   rsmt2d.Axis
	index  uint
	pushed int                                   // cells pushed that match the table
	cpu    *wrapper.ErasuredNamespacedMerkleTree // the reference tree, once a cell differs
}

func (tr *rootTree) cell(j int) []byte {
	if tr.axis == rsmt2d.Row {
		return tr.t.Cells[int(tr.index)*tr.t.Width+j]
	}
	return tr.t.Cells[j*tr.t.Width+int(tr.index)]
}

// reference builds the reference tree over the matching cells pushed so far.
func (tr *rootTree) reference() error {
	t := wrapper.NewErasuredNamespacedMerkleTree(uint64(tr.t.Width/2), tr.index)
	tr.cpu = &t
	for j := 0; j < tr.pushed; j++ {
		if err := tr.cpu.Push(tr.cell(j)); err != nil {
			return err
		}
	}
	return nil
}

// Push keeps wrapper.Push's argument checks and messages (nmt_wrapper.go:93-99).
func (tr *rootTree) Push(data []byte) error {
	if tr.cpu != nil {
		return tr.cpu.Push(data)
	}
	w := tr.t.Width
	if int(tr.index)+1 > w || tr.pushed+1 > w {
		return fmt.Errorf("pushed past predetermined square size: boundary at %d index at %d %d", w, tr.index,
			tr.pushed)
	}
	if len(data) < appconsts.NamespaceSize {
		return fmt.Errorf("data is too short to contain namespace ID")
	}
	if bytes.Equal(data, tr.cell(tr.pushed)) {
		tr.pushed++
		return nil
	}
	if err := tr.reference(); err != nil {
		return err
	}
	return tr.cpu.Push(data)
}

func (tr *rootTree) Root() ([]byte, error) {
	if tr.cpu == nil && tr.pushed == tr.t.Width {
		if tr.axis == rsmt2d.Row {
			return tr.t.Rows[tr.index], nil
		}
		return tr.t.Cols[tr.index], nil
	}
	if tr.cpu == nil { // a partial axis: the device holds only full-axis roots
		if err := tr.reference(); err != nil {
			return nil, err
		}
	}
	return tr.cpu.Root()
}
