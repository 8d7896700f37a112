package celestiaeds

/*
#include <stdlib.h>
#include "celestia_eds.h"
*/
import "C"

import (
	"fmt"
	"sort"
	"unsafe"

	"github.com/celestiaorg/celestia-app/v3/pkg/wrapper"
	"github.com/celestiaorg/rsmt2d"
)

// Group is several devices driven by one Go process through the library's multi-GPU entry
// points (include/celestia_eds.h, "multi-GPU" section): one Context per device, rank order =
// slice order. The collectives (the row-sharded square's all-to-all transpose and record
// all-gather) are RCCL calls the library issues itself, so no torchrun or MPI launcher is
// involved: the node process that calls da.ExtendShares (pkg/da/data_availability_header.go:65)
// reaches configs 3 and 4 of BASELINE.json directly.
type Group struct {
	Ctxs []*Context
}

// NewGroup opens one Context per device.
func NewGroup(devices []int) (*Group, error) {
	g := &Group{}
	for _, d := range devices {
		c, err := NewContext(d)
		if err != nil {
			g.Close()
			return nil, err
		}
		g.Ctxs = append(g.Ctxs, c)
	}
	return g, nil
}

func (g *Group) Close() {
	for _, c := range g.Ctxs {
		c.Close()
	}
	g.Ctxs = nil
}

// handles returns the cel_ctx pointers in C memory (cgo may not pass a Go slice of C
// pointers that the callee keeps) and a release func. Every distinct Context's lock is held
// until release (the library call uses all of them), taken in one fixed order (by the
// cel_ctx address, whatever the slice order), so two Groups sharing Contexts in different
// orders cannot deadlock.
func (g *Group) handles() (**C.cel_ctx, func()) {
	n := len(g.Ctxs)
	arr := (**C.cel_ctx)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0)))))
	s := unsafe.Slice(arr, n)
	seen := map[*Context]bool{}
	var distinct []*Context
	for i, c := range g.Ctxs {
		s[i] = c.ctx
		if !seen[c] {
			seen[c] = true
			distinct = append(distinct, c)
		}
	}
	sort.Slice(distinct, func(a, b int) bool {
		return uintptr(unsafe.Pointer(distinct[a].ctx)) < uintptr(unsafe.Pointer(distinct[b].ctx))
	})
	for _, c := range distinct {
		c.mu.Lock()
	}
	return arr, func() {
		for i := len(distinct) - 1; i >= 0; i-- {
			distinct[i].mu.Unlock()
		}
		C.free(unsafe.Pointer(arr))
	}
}

// ExtendSquare is (*Context).ExtendSquare for one square row-sharded over the group
// (cel_extend_sharded): k = 256 or 512 (Leopard GF(2^16); the e2e big-block size,
// test/e2e/benchmark/throughput.go:49), the group's size a power of two <= k. The ODS goes
// up split by rows, one block per device; only the parity cells come back (Q0 of the
// imported square points at the input shares) together with all 4k roots, and the square
// is imported with a RootTable constructor like the single-device path. Other widths, other
// codecs and other share sizes go to the reference call, as in (*Context).ExtendSquare.
func (g *Group) ExtendSquare(shares [][]byte, codec rsmt2d.Codec) (*rsmt2d.ExtendedDataSquare, error) {
	n := len(shares)
	if n == 0 || n&(n-1) != 0 {
		return nil, fmt.Errorf("number of shares is not a power of 2: got %d", n)
	}
	k := squareWidth(n)
	if (k != 256 && k != 512) || !deviceCodec(codec) || !deviceShares(shares) || len(g.Ctxs) == 0 {
		if len(g.Ctxs) > 0 && deviceCodec(codec) && deviceShares(shares) {
			return g.Ctxs[0].ExtendSquare(shares, codec) // a width the sharded mode does not cover
		}
		return rsmt2d.ComputeExtendedDataSquare(shares, codec, wrapper.NewConstructor(uint64(k)))
	}
	w := 2 * k
	flat := make([]byte, w*w*ShareSize)
	rr := make([]byte, w*NmtNodeSize)
	cr := make([]byte, w*NmtNodeSize)
	dah := make([]byte, 32)
	arr, release := g.handles()
	// the first Context's page-locked staging (its lock is held): the per-device row blocks
	// go up by DMA from page-locked memory
	buf, rel := g.Ctxs[0].stagedLocked(shares)
	if rel != nil {
		defer rel()
	}
	st := C.cel_extend_sharded(arr, C.uint32_t(len(g.Ctxs)), (*C.uint8_t)(buf), C.uint32_t(k), ShareSize,
		(*C.uint8_t)(unsafe.Pointer(&flat[0])), (*C.uint8_t)(unsafe.Pointer(&rr[0])),
		(*C.uint8_t)(unsafe.Pointer(&cr[0])), (*C.uint8_t)(unsafe.Pointer(&dah[0])), flagOrder|flagParity)
	err := g.Ctxs[0].errLocked(st) // reads ctxs[0]'s message while its lock is held
	release()
	if err != nil {
		return nil, err
	}
	rows := make([][]byte, w)
	cols := make([][]byte, w)
	for i := 0; i < w; i++ {
		rows[i] = rr[i*NmtNodeSize : (i+1)*NmtNodeSize]
		cols[i] = cr[i*NmtNodeSize : (i+1)*NmtNodeSize]
	}
	cells := make([][]byte, w*w)
	for i := range cells {
		if r, col := i/w, i%w; r < k && col < k {
			cells[i] = shares[r*k+col]
		} else {
			cells[i] = flat[i*ShareSize : (i+1)*ShareSize]
		}
	}
	table := &RootTable{Rows: rows, Cols: cols, Cells: cells, Width: w}
	return rsmt2d.ImportExtendedDataSquare(cells, codec, table.NewTree)
}

// DataAvailabilityHeaders is ComputeDataAvailabilityHeader (INTEGRATION.md §2) for a
// batch of independent squares of one width (block replay, config 4), split over the
// group's devices, one host thread per device inside the library
// (cel_extend_batch_multi): roots only come back. Each element of squares is one block's
// ODS as da.ExtendShares receives it.
func (g *Group) DataAvailabilityHeaders(squares [][][]byte) (rowRoots, colRoots [][][]byte, err error) {
	if len(squares) == 0 || len(g.Ctxs) == 0 {
		return nil, nil, nil
	}
	n := len(squares[0])
	if n == 0 || n&(n-1) != 0 {
		return nil, nil, fmt.Errorf("number of shares is not a power of 2: got %d", n)
	}
	for _, sq := range squares {
		if len(sq) != n || !deviceShares(sq) {
			return nil, nil, &StatusError{Status: int(C.CEL_EINVAL),
				Msg: "every square of a batch needs the same number of 512-byte shares"}
		}
	}
	k := squareWidth(n)
	m := len(squares)
	all := make([][]byte, 0, m*n)
	for _, sq := range squares {
		all = append(all, sq...)
	}
	w := 2 * k
	rr := make([]byte, m*w*NmtNodeSize)
	cr := make([]byte, m*w*NmtNodeSize)
	dah := make([]byte, m*32)
	arr, release := g.handles()
	buf, rel := g.Ctxs[0].stagedLocked(all) // page-locked: every chunk's upload is a plain DMA
	if rel != nil {
		defer rel()
	}
	st := C.cel_extend_batch_multi(arr, C.uint32_t(len(g.Ctxs)), (*C.uint8_t)(buf), C.uint32_t(m), C.uint32_t(k),
		ShareSize, nil, (*C.uint8_t)(unsafe.Pointer(&rr[0])), (*C.uint8_t)(unsafe.Pointer(&cr[0])),
		(*C.uint8_t)(unsafe.Pointer(&dah[0])), nil, flagOrder)
	err = g.Ctxs[0].errLocked(st)
	release()
	if tooBig(err) { // k > 512: the reference path, square by square
		for _, sq := range squares {
			r, c, rerr := g.Ctxs[0].DataAvailabilityHeader(sq, refCodec)
			if rerr != nil {
				return nil, nil, rerr
			}
			rowRoots = append(rowRoots, r)
			colRoots = append(colRoots, c)
		}
		return rowRoots, colRoots, nil
	}
	if err != nil {
		return nil, nil, err
	}
	for j := 0; j < m; j++ {
		r := make([][]byte, w)
		c := make([][]byte, w)
		for i := 0; i < w; i++ {
			off := (j*w + i) * NmtNodeSize
			r[i] = rr[off : off+NmtNodeSize]
			c[i] = cr[off : off+NmtNodeSize]
		}
		rowRoots = append(rowRoots, r)
		colRoots = append(colRoots, c)
	}
	return rowRoots, colRoots, nil
}
