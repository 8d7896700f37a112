// Package celestiaeds binds libcelestia_eds.so (MI355X / gfx950) behind the
// reference's own Go surface: rsmt2d's Codec, TreeConstructorFn / Tree and
// ErrByzantineData types (rsmt2d v0.14.0, go.mod:13). It is the cgo stub a
// celestia-app maintainer would add as pkg/celestiaeds of module
// github.com/celestiaorg/celestia-app/v3; this repository's build image has no Go
// toolchain, so it is not compiled here (parity is established through the C ABI
// tests, which drive the same entry points).
//
// Replaces, without changing signatures:
//   pkg/da/data_availability_header.go:65  da.ExtendShares (ExtendSquare below)
//   pkg/da/data_availability_header.go:44  da.NewDataAvailabilityHeader (roots precomputed, RootTable)
//   pkg/appconsts/global_consts.go:92       appconsts.DefaultCodec (Codec, an rsmt2d.Codec)
//   rsmt2d ExtendedDataSquare.Repair        (Context.Repair, used by celestia-node)
package celestiaeds

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../celestia-app_amd -lcelestia_eds -Wl,-rpath,${SRCDIR}/../../celestia-app_amd
#include <stdlib.h>
#include "celestia_eds.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"sync"
	"unsafe"

	"github.com/celestiaorg/celestia-app/v3/pkg/appconsts"
	"github.com/celestiaorg/celestia-app/v3/pkg/wrapper"
	"github.com/celestiaorg/rsmt2d"
)

const (
	ShareSize    = C.CEL_SHARE_SIZE
	NmtNodeSize  = C.CEL_NMT_NODE_SIZE
	flagOrder    = C.CEL_FLAG_ORDER_CHECK
	flagParity   = C.CEL_FLAG_PARITY_ONLY
)

// Status codes map onto the reference's Go errors (include/celestia_eds.h):
// CEL_EBYZANTINE -> *rsmt2d.ErrByzantineData, CEL_EUNREPAIRABLE ->
// rsmt2d.ErrUnrepairableDataSquare, the rest -> a *StatusError carrying the reference's
// message (errors.Is(err, ErrNotPow2) for CEL_ENOTPOW2).
var ErrNotPow2 = errors.New("number of shares is not a power of 2")

// StatusError is a failing cel_* call: its status code and cel_last_error's message.
type StatusError struct {
	Status int
	Msg    string
}

func (e *StatusError) Error() string { return e.Msg }

func (e *StatusError) Unwrap() error {
	if e.Status == C.CEL_ENOTPOW2 {
		return ErrNotPow2
	}
	return nil
}

// tooBig reports whether err is CEL_ETOOBIG: a square or codeword wider than the device
// path. Those calls are answered by the reference path instead (INTEGRATION.md §1).
func tooBig(err error) bool {
	var se *StatusError
	return errors.As(err, &se) && se.Status == C.CEL_ETOOBIG
}

// deviceCodec reports whether codec computes what the device computes: Leopard parity
// (rsmt2d.NewLeoRSCodec, appconsts.DefaultCodec at pkg/appconsts/global_consts.go:92;
// cel_codec_name() is "Leopard"). Any other rsmt2d.Codec gets the reference path, so its
// parity and roots are that codec's.
func deviceCodec(codec rsmt2d.Codec) bool {
	return codec != nil && codec.Name() == C.GoString(C.cel_codec_name())
}

// deviceShares reports whether every share is appconsts.ShareSize bytes, the only share
// size the device path takes (the C ABI receives n and the size, never the lengths). Other
// lengths go to rsmt2d, which extends any equal, 64-byte-multiple chunk size and returns
// its own error for the rest.
func deviceShares(shares [][]byte) bool {
	for _, s := range shares {
		if len(s) != ShareSize {
			return false
		}
	}
	return true
}

func squareWidth(n int) int {
	k := 1
	for k*k < n {
		k <<= 1
	}
	return k
}

type Context struct {
	mu  sync.Mutex
	ctx *C.cel_ctx
	// Page-locked staging for an ODS (cel_host_alloc, grown on demand, used under mu). The
	// library's one-square path reads page-locked input straight over PCIe (k <= 128) or
	// uploads it in chunks beside the row pass (k = 512); from ordinary memory the same
	// header takes 5-10 % longer (profiles/r5_header_pageable_ods.txt).
	stage    unsafe.Pointer
	stageLen int
}

// maxKeptStage is the most page-locked staging a Context keeps between calls: one k = 512
// ODS (512 x 512 x 512 B). Larger batches stage in a buffer of their own, freed after the call.
const maxKeptStage = 512 * 512 * ShareSize

// stagedLocked copies shares into the page-locked staging buffer and returns it, or a
// buffer of this call's own (release != nil: the caller frees it) for a batch above
// maxKeptStage or when page-locked memory is not to be had. The caller holds c.mu.
func (c *Context) stagedLocked(shares [][]byte) (buf unsafe.Pointer, release func()) {
	need := len(shares) * ShareSize
	if need > maxKeptStage {
		// a batch beyond one k = 512 ODS: page-locked for this call only, so a replay of many
		// squares does not leave that much host memory pinned for the Context's lifetime
		buf = C.cel_host_alloc(C.size_t(need))
		if buf != nil {
			release = func() { C.cel_host_free(buf) }
		} else {
			buf = C.malloc(C.size_t(need))
			release = func() { C.free(buf) }
		}
		copyShares(unsafe.Slice((*byte)(buf), need), shares)
		return buf, release
	}
	if c.stageLen < need {
		if c.stage != nil {
			C.cel_host_free(c.stage)
		}
		c.stage, c.stageLen = C.cel_host_alloc(C.size_t(need)), need
		if c.stage == nil {
			c.stageLen = 0
		}
	}
	buf = c.stage
	if buf == nil {
		buf = C.malloc(C.size_t(need))
		release = func() { C.free(buf) }
	}
	dst := unsafe.Slice((*byte)(buf), need)
	copyShares(dst, shares)
	return buf, release
}

// copyShares flattens shares into dst, split over up to 8 goroutines for a large square
// (one core copies ~8 MiB, a k = 128 ODS, in about as long as the device takes for the
// whole header).
func copyShares(dst []byte, shares [][]byte) {
	parts := runtime.GOMAXPROCS(0)
	if parts > 8 {
		parts = 8
	}
	if len(dst) < 4<<20 || parts < 2 {
		for i, s := range shares {
			copy(dst[i*ShareSize:], s)
		}
		return
	}
	var wg sync.WaitGroup
	per := (len(shares) + parts - 1) / parts
	for lo := 0; lo < len(shares); lo += per {
		hi := lo + per
		if hi > len(shares) {
			hi = len(shares)
		}
		wg.Add(1)
		go func(lo, hi int) {
			defer wg.Done()
			for i := lo; i < hi; i++ {
				copy(dst[i*ShareSize:], shares[i])
			}
		}(lo, hi)
	}
	wg.Wait()
}

func NewContext(device int) (*Context, error) {
	var c *C.cel_ctx
	if st := C.cel_ctx_create(C.int(device), &c); st != C.CEL_OK {
		return nil, fmt.Errorf("cel_ctx_create: %s", C.GoString(C.cel_strerror(st)))
	}
	return &Context{ctx: c}, nil
}

func (c *Context) Close() {
	c.mu.Lock()
	defer c.mu.Unlock()
	if c.stage != nil {
		C.cel_host_free(c.stage)
		c.stage, c.stageLen = nil, 0
	}
	C.cel_ctx_destroy(c.ctx)
}

// call runs f (a cel_* call on c.ctx) under c.mu and turns its status into an error,
// reading cel_last_error before the lock is released (another goroutine's call on the
// same ctx would overwrite it).
func (c *Context) call(f func() C.cel_status) error {
	c.mu.Lock()
	defer c.mu.Unlock()
	return c.errLocked(f())
}

func (c *Context) errLocked(st C.cel_status) error {
	if st == C.CEL_OK {
		return nil
	}
	if st == C.CEL_EUNREPAIRABLE {
		return rsmt2d.ErrUnrepairableDataSquare
	}
	return &StatusError{Status: int(st), Msg: C.GoString(C.cel_last_error(c.ctx))}
}

// ExtendShares is the device pass behind da.ExtendShares: the [][]byte ODS is copied
// into one contiguous buffer (cgo may not retain Go pointers), extended on the GPU, and
// the whole flattened EDS (Q0 included) plus all 4k roots and the DAH hash come back in
// one call. A caller can wrap flat with rsmt2d.ImportExtendedDataSquare(cells of flat,
// codec, (&RootTable{...}).NewTree). ExtendSquare does that with less PCIe traffic.
func (c *Context) ExtendShares(shares [][]byte) (flat []byte, rowRoots, colRoots [][]byte, dah []byte, err error) {
	if !deviceShares(shares) {
		return nil, nil, nil, nil, &StatusError{Status: C.CEL_ECHUNK,
			Msg: fmt.Sprintf("every share must be %d bytes on the device path", ShareSize)}
	}
	return c.extend(shares, flagOrder)
}

// extend runs cel_extend_shares with flags. With flagParity only the parity cells cross
// PCIe and flat's Q0 cells stay zero: the caller points them at the input shares.
func (c *Context) extend(shares [][]byte, flags C.uint32_t) (flat []byte, rowRoots, colRoots [][]byte, dah []byte,
	err error) {
	n := len(shares)
	w := 2 * squareWidth(n)
	flat = make([]byte, w*w*ShareSize)
	rr := make([]byte, w*NmtNodeSize)
	cr := make([]byte, w*NmtNodeSize)
	dah = make([]byte, 32)
	c.mu.Lock()
	buf, release := c.stagedLocked(shares)
	err = c.errLocked(C.cel_extend_shares(c.ctx, (*C.uint8_t)(buf), C.uint32_t(n), ShareSize,
		(*C.uint8_t)(unsafe.Pointer(&flat[0])), (*C.uint8_t)(unsafe.Pointer(&rr[0])),
		(*C.uint8_t)(unsafe.Pointer(&cr[0])), (*C.uint8_t)(unsafe.Pointer(&dah[0])), flags))
	c.mu.Unlock()
	if release != nil {
		release()
	}
	if err != nil {
		return nil, nil, nil, nil, err
	}
	for i := 0; i < w; i++ {
		rowRoots = append(rowRoots, rr[i*NmtNodeSize:(i+1)*NmtNodeSize])
		colRoots = append(colRoots, cr[i*NmtNodeSize:(i+1)*NmtNodeSize])
	}
	return flat, rowRoots, colRoots, dah, nil
}

// ExtendSquare is da.ExtendShares on the device (data_availability_header.go:65-75):
// the same power-of-two check and error, then one device pass, and an
// *rsmt2d.ExtendedDataSquare imported with a RootTable constructor, so
// da.NewDataAvailabilityHeader's eds.RowRoots()/ColRoots() return the device roots.
// A square wider than the device path (CEL_ETOOBIG: k > 512), and a codec other than
// Leopard, are extended by the reference call itself, rsmt2d.ComputeExtendedDataSquare
// with wrapper.NewConstructor, exactly as data_availability_header.go:74 does: the domain
// and the codec stay the reference's.
func (c *Context) ExtendSquare(shares [][]byte, codec rsmt2d.Codec) (*rsmt2d.ExtendedDataSquare, error) {
	if n := len(shares); n == 0 || n&(n-1) != 0 {
		return nil, fmt.Errorf("number of shares is not a power of 2: got %d", n)
	}
	if !deviceCodec(codec) || !deviceShares(shares) {
		return rsmt2d.ComputeExtendedDataSquare(shares, codec, wrapper.NewConstructor(uint64(squareWidth(len(shares)))))
	}
	flat, rr, cr, _, err := c.extend(shares, flagOrder|flagParity)
	if tooBig(err) {
		return rsmt2d.ComputeExtendedDataSquare(shares, codec, wrapper.NewConstructor(uint64(squareWidth(len(shares)))))
	}
	if err != nil {
		return nil, err
	}
	w := len(rr)
	k := w / 2
	cells := make([][]byte, w*w)
	for i := range cells {
		if r, col := i/w, i%w; r < k && col < k {
			cells[i] = shares[r*k+col] // Q0: the ODS itself (not copied back)
		} else {
			cells[i] = flat[i*ShareSize : (i+1)*ShareSize]
		}
	}
	table := &RootTable{Rows: rr, Cols: cr, Cells: cells, Width: w}
	return rsmt2d.ImportExtendedDataSquare(cells, codec, table.NewTree)
}

// DataAvailabilityHeader is da.NewDataAvailabilityHeader(da.ExtendShares(shares)) for the
// callers that keep only the header: app/prepare_proposal.go:61-92 and
// app/process_proposal.go:138-156 use nothing but dah.Hash() ("the eds is not returned
// here"). One device pass with no EDS copied back (cel_extend_shares, eds_out = NULL): 8 MiB
// up and 46 KB of roots down for k = 128 instead of 8 MiB up and 24 MiB down. Outside the
// device's domain (CEL_ETOOBIG), or with a codec other than Leopard, the reference computes
// it: rsmt2d.ComputeExtendedDataSquare with wrapper.NewConstructor, then the square's
// RowRoots / ColRoots.
func (c *Context) DataAvailabilityHeader(shares [][]byte, codec rsmt2d.Codec) (rowRoots, colRoots [][]byte, err error) {
	n := len(shares)
	if n == 0 || n&(n-1) != 0 {
		return nil, nil, fmt.Errorf("number of shares is not a power of 2: got %d", n)
	}
	k := squareWidth(n)
	reference := func() ([][]byte, [][]byte, error) {
		eds, cerr := rsmt2d.ComputeExtendedDataSquare(shares, codec, wrapper.NewConstructor(uint64(k)))
		if cerr != nil {
			return nil, nil, cerr
		}
		rows, rerr := eds.RowRoots()
		if rerr != nil {
			return nil, nil, rerr
		}
		cols, cerr := eds.ColRoots()
		return rows, cols, cerr
	}
	if !deviceCodec(codec) || !deviceShares(shares) {
		return reference()
	}
	w := 2 * k
	rr := make([]byte, w*NmtNodeSize)
	cr := make([]byte, w*NmtNodeSize)
	dah := make([]byte, 32)
	c.mu.Lock()
	buf, release := c.stagedLocked(shares)
	err = c.errLocked(C.cel_extend_shares(c.ctx, (*C.uint8_t)(buf), C.uint32_t(n), ShareSize, nil,
		(*C.uint8_t)(unsafe.Pointer(&rr[0])), (*C.uint8_t)(unsafe.Pointer(&cr[0])),
		(*C.uint8_t)(unsafe.Pointer(&dah[0])), flagOrder))
	c.mu.Unlock()
	if release != nil {
		release()
	}
	if tooBig(err) {
		return reference()
	}
	if err != nil {
		return nil, nil, err
	}
	for i := 0; i < w; i++ {
		rowRoots = append(rowRoots, rr[i*NmtNodeSize:(i+1)*NmtNodeSize])
		colRoots = append(colRoots, cr[i*NmtNodeSize:(i+1)*NmtNodeSize])
	}
	return rowRoots, colRoots, nil
}

// Codec implements rsmt2d.Codec (Encode/Decode/MaxChunks/Name/ValidateChunkSize) on
// the device; rsmt2d's per-axis calls pay one launch each, so the square path above
// is the fast path and this exists for API completeness (e.g. Repair from celestia-node).
// MaxChunks is the reference's 32768^2; codewords wider than the device kernels (encode
// n > 2048 data shards, decode n > 1024: CEL_ETOOBIG) go to the reference LeoRSCodec
// (appconsts.DefaultCodec, global_consts.go:92), so every input the reference accepts
// is accepted here with the reference's result. So are the inputs the C ABI cannot be
// handed (no shards, no bytes, shards of unequal lengths, an odd codeword): the reference
// codec returns its own error for them.
type Codec struct{ C *Context }

var refCodec = appconsts.DefaultCodec()

var _ rsmt2d.Codec = Codec{}

func (cd Codec) Name() string    { return C.GoString(C.cel_codec_name()) }
func (cd Codec) MaxChunks() int  { return int(C.cel_codec_max_chunks()) }
func (cd Codec) ValidateChunkSize(n int) error {
	if C.cel_codec_validate_chunk_size(C.uint32_t(n)) != C.CEL_OK {
		return fmt.Errorf("chunkSize %d must be a multiple of 64 bytes", n)
	}
	return nil
}

func (cd Codec) Encode(data [][]byte) ([][]byte, error) {
	if len(data) == 0 || len(data[0]) == 0 {
		return refCodec.Encode(data)
	}
	n, l := len(data), len(data[0])
	for _, d := range data {
		if len(d) != l {
			return refCodec.Encode(data)
		}
	}
	in := C.malloc(C.size_t(n * l))
	out := C.malloc(C.size_t(n * l))
	defer C.free(in)
	defer C.free(out)
	src := unsafe.Slice((*byte)(in), n*l)
	for i, d := range data {
		copy(src[i*l:], d)
	}
	if err := cd.C.call(func() C.cel_status {
		return C.cel_codec_encode(cd.C.ctx, (*C.uint8_t)(in), C.uint32_t(n), C.uint32_t(l), (*C.uint8_t)(out))
	}); tooBig(err) {
		return refCodec.Encode(data)
	} else if err != nil {
		return nil, err
	}
	par := unsafe.Slice((*byte)(out), n*l)
	res := make([][]byte, n)
	for i := range res {
		res[i] = append([]byte(nil), par[i*l:(i+1)*l]...)
	}
	return res, nil
}

func (cd Codec) Decode(shards [][]byte) ([][]byte, error) {
	n2 := len(shards)
	l := 0
	for _, s := range shards {
		if s != nil {
			l = len(s)
			break
		}
	}
	if n2 == 0 || n2%2 != 0 || l == 0 {
		return refCodec.Decode(shards)
	}
	for _, s := range shards {
		if s != nil && len(s) != l {
			return refCodec.Decode(shards)
		}
	}
	buf := C.malloc(C.size_t(n2 * l))
	pres := C.malloc(C.size_t(n2))
	defer C.free(buf)
	defer C.free(pres)
	b := unsafe.Slice((*byte)(buf), n2*l)
	p := unsafe.Slice((*byte)(pres), n2)
	for i, s := range shards {
		if s != nil {
			copy(b[i*l:], s)
			p[i] = 1
		} else {
			p[i] = 0
		}
	}
	if err := cd.C.call(func() C.cel_status {
		return C.cel_codec_decode(cd.C.ctx, (*C.uint8_t)(buf), (*C.uint8_t)(pres), C.uint32_t(n2/2), C.uint32_t(l))
	}); tooBig(err) {
		return refCodec.Decode(shards)
	} else if err != nil {
		return nil, err
	}
	out := make([][]byte, n2)
	for i := range out {
		out[i] = append([]byte(nil), b[i*l:(i+1)*l]...)
	}
	return out, nil
}

// SquareConstruct wraps cel_square_construct: go-square square.Construct (greedy =
// false) or square.Build (greedy = true). It returns the ODS shares and, for Build,
// which txs were kept. Host-only: no device work.
func SquareConstruct(txs [][]byte, maxSquareSize, subtreeRootThreshold int, greedy bool) ([][]byte, []bool, error) {
	total := 0
	for _, t := range txs {
		total += len(t)
	}
	buf := C.malloc(C.size_t(total + 1))
	lens := C.malloc(C.size_t(4 * (len(txs) + 1)))
	inc := C.malloc(C.size_t(len(txs) + 1))
	defer C.free(buf)
	defer C.free(lens)
	defer C.free(inc)
	b := unsafe.Slice((*byte)(buf), total+1)
	l := unsafe.Slice((*C.uint32_t)(lens), len(txs)+1)
	off := 0
	for i, t := range txs {
		copy(b[off:], t)
		l[i] = C.uint32_t(len(t))
		off += len(t)
	}
	g := C.uint32_t(0)
	if greedy {
		g = 1
	}
	var k C.uint32_t
	st := C.cel_square_construct((*C.uint8_t)(buf), (*C.uint32_t)(lens), C.uint32_t(len(txs)),
		C.uint32_t(maxSquareSize), C.uint32_t(subtreeRootThreshold), g, nil, 0, &k, (*C.uint8_t)(inc))
	if st != 0 {
		return nil, nil, fmt.Errorf("%s", C.GoString(C.cel_square_last_error()))
	}
	n := int(k) * int(k)
	out := C.malloc(C.size_t(n * C.CEL_SHARE_SIZE))
	defer C.free(out)
	st = C.cel_square_construct((*C.uint8_t)(buf), (*C.uint32_t)(lens), C.uint32_t(len(txs)),
		C.uint32_t(maxSquareSize), C.uint32_t(subtreeRootThreshold), g, (*C.uint8_t)(out), C.uint32_t(n), &k,
		(*C.uint8_t)(inc))
	if st != 0 {
		return nil, nil, fmt.Errorf("%s", C.GoString(C.cel_square_last_error()))
	}
	o := unsafe.Slice((*byte)(out), n*C.CEL_SHARE_SIZE)
	shares := make([][]byte, n)
	for i := range shares {
		shares[i] = append([]byte(nil), o[i*C.CEL_SHARE_SIZE:(i+1)*C.CEL_SHARE_SIZE]...)
	}
	kept := make([]bool, len(txs))
	iv := unsafe.Slice((*byte)(inc), len(txs)+1)
	for i := range kept {
		kept[i] = iv[i] != 0 // 1 = normal tx kept, 2 = blob tx kept
	}
	return shares, kept, nil
}

// GetCommitment wraps cel_get_commitment (pkg/inclusion.GetCommitment without the
// EDSSubTreeRootCacher: the device hashes the rows' trees). eds: the flattened
// 2k x 2k square.
func (c *Context) GetCommitment(eds []byte, k, start, blobShareLen, subtreeRootThreshold int) ([]byte, error) {
	buf := C.CBytes(eds)
	defer C.free(buf)
	out := make([]byte, 32)
	if err := c.call(func() C.cel_status {
		return C.cel_get_commitment(c.ctx, (*C.uint8_t)(buf), C.uint32_t(k), C.CEL_SHARE_SIZE, C.uint32_t(start),
			C.uint32_t(blobShareLen), C.uint32_t(subtreeRootThreshold), (*C.uint8_t)(unsafe.Pointer(&out[0])))
	}); err != nil {
		return nil, err
	}
	return out, nil
}

// ProveRange is ErasuredNamespacedMerkleTree.ProveRange (pkg/wrapper/nmt_wrapper.go:127-130)
// for a full axis: cells are the axis's 2k shares (what the wrapper tree was pushed),
// axisIndex its index; the device hashes every node of the axis tree (cel_axis_tree) and
// cel_nmt_prove_range picks the proof nodes of [start, end), which
// nmt.NewInclusionProof(start, end, nodes, true) turns into the nmt.Proof the wrapper
// returns (IgnoreMaxNamespace, as wrapper.NewErasuredNamespacedMerkleTree sets it).
func (c *Context) ProveRange(cells [][]byte, k, axisIndex, start, end int) ([][]byte, error) {
	// Go ints would wrap through C.uint32_t: reject what the reference tree would never see
	if k <= 0 || axisIndex < 0 || axisIndex >= 2*k || start < 0 || end < 0 {
		return nil, &StatusError{Status: int(C.CEL_EINVAL),
			Msg: fmt.Sprintf("invalid ProveRange arguments: k=%d axisIndex=%d range [%d, %d)", k, axisIndex, start, end)}
	}
	if len(cells) != 2*k || !deviceShares(cells) {
		return nil, &StatusError{Status: int(C.CEL_EINVAL), Msg: "ProveRange needs the axis's 2k shares of 512 bytes"}
	}
	flat := make([]byte, 0, 2*k*ShareSize)
	for _, s := range cells {
		flat = append(flat, s...)
	}
	tree := make([]byte, (4*k-1)*NmtNodeSize)
	if err := c.call(func() C.cel_status {
		return C.cel_axis_tree(c.ctx, (*C.uint8_t)(unsafe.Pointer(&flat[0])), C.uint32_t(k), C.uint32_t(axisIndex),
			C.CEL_SHARE_SIZE, (*C.uint8_t)(unsafe.Pointer(&tree[0])))
	}); err != nil {
		return nil, err
	}
	var n C.uint32_t
	if st := C.cel_nmt_prove_range((*C.uint8_t)(unsafe.Pointer(&tree[0])), C.uint32_t(2*k), C.uint32_t(start),
		C.uint32_t(end), nil, &n); st != C.CEL_OK {
		return nil, &StatusError{Status: int(st), Msg: fmt.Sprintf("invalid range [%d, %d) over %d leaves", start, end, 2*k)}
	}
	out := make([]byte, int(n)*NmtNodeSize)
	if n > 0 {
		C.cel_nmt_prove_range((*C.uint8_t)(unsafe.Pointer(&tree[0])), C.uint32_t(2*k), C.uint32_t(start),
			C.uint32_t(end), (*C.uint8_t)(unsafe.Pointer(&out[0])), &n)
	}
	nodes := make([][]byte, int(n))
	for i := range nodes {
		nodes[i] = out[i*NmtNodeSize : (i+1)*NmtNodeSize]
	}
	return nodes, nil
}

// Repair wraps cel_repair, the device pass behind rsmt2d.ExtendedDataSquare.Repair
// (rsmt2d v0.14.0 extendeddatacrossword.go): flat is the flattened 2k x 2k square
// (missing cells may hold anything), present[i] != 0 marks known cells. On success
// every cell of flat is filled in place. Errors are rsmt2d's: *rsmt2d.ErrByzantineData
// with the byzantine axis's Shares (nil where the repair did not know the cell, the
// shares a celestia-node bad-encoding fraud proof is built from), the plain "bad root
// input" error of preRepairSanityCheck, or rsmt2d.ErrUnrepairableDataSquare. On an
// error present[] is left as the mask the partially repaired flat is valid under.
// Squares wider than the device path (CEL_ETOOBIG, k > 512) are repaired by rsmt2d itself;
// if that fallback fails, flat and present[] are left exactly as the caller passed them
// (rsmt2d fills new cell slices, never the known cells it imported from flat).
func (c *Context) Repair(flat, present []byte, k int, rowRoots, colRoots [][]byte) error {
	w := 2 * k
	rr := make([]byte, 0, w*NmtNodeSize)
	cr := make([]byte, 0, w*NmtNodeSize)
	for i := 0; i < w; i++ {
		rr = append(rr, rowRoots[i]...)
		cr = append(cr, colRoots[i]...)
	}
	byzShares := make([]byte, w*ShareSize)
	byzPresent := make([]byte, w)
	var axis, index C.int32_t
	var st C.cel_status
	err := c.call(func() C.cel_status {
		st = C.cel_repair(c.ctx, (*C.uint8_t)(unsafe.Pointer(&flat[0])), (*C.uint8_t)(unsafe.Pointer(&present[0])),
			C.uint32_t(k), ShareSize, (*C.uint8_t)(unsafe.Pointer(&rr[0])), (*C.uint8_t)(unsafe.Pointer(&cr[0])),
			&axis, &index, (*C.uint8_t)(unsafe.Pointer(&byzShares[0])), (*C.uint8_t)(unsafe.Pointer(&byzPresent[0])))
		return st
	})
	if tooBig(err) { // k > 512: rsmt2d's own Repair over the same cells
		cells := make([][]byte, w*w)
		for i := range cells {
			if present[i] != 0 {
				cells[i] = flat[i*ShareSize : (i+1)*ShareSize]
			}
		}
		eds, ierr := rsmt2d.ImportExtendedDataSquare(cells, appconsts.DefaultCodec(), wrapper.NewConstructor(uint64(k)))
		if ierr != nil {
			return ierr
		}
		if rerr := eds.Repair(rowRoots, colRoots); rerr != nil {
			return rerr
		}
		for i := range cells {
			copy(flat[i*ShareSize:(i+1)*ShareSize], eds.GetCell(uint(i/w), uint(i%w)))
			present[i] = 1
		}
		return nil
	}
	if st == C.CEL_EBYZANTINE {
		shares := make([][]byte, w)
		for j := range shares {
			if byzPresent[j] != 0 {
				shares[j] = byzShares[j*ShareSize : (j+1)*ShareSize]
			}
		}
		return &rsmt2d.ErrByzantineData{Axis: rsmt2d.Axis(axis), Index: uint(index), Shares: shares}
	}
	return err
}

// PinnedBuffer returns page-locked host memory (cel_host_alloc) for the flattened
// ODS / EDS buffers of ExtendShares-style calls; free it with FreePinned.
func PinnedBuffer(n int) []byte {
	p := C.cel_host_alloc(C.size_t(n))
	if p == nil {
		return nil
	}
	return unsafe.Slice((*byte)(p), n)
}

func FreePinned(b []byte) {
	if len(b) > 0 {
		C.cel_host_free(unsafe.Pointer(&b[0]))
	}
}
