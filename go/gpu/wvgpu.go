//go:build rocm

// Package gpu binds libwvgpu.so, the MI355X (gfx950) backend of Weaviate's
// flat / BQ / PQ vector-scoring hot path, through its C ABI (include/wvgpu.h).
// It sits in the reference tree at adapters/repos/db/vector/gpu and is built
// only with `go build -tags rocm`; the default pure-Go build never sees it.
//
// Every function maps one-to-one onto a wvg_* entry point (the Go symbol each
// one replaces is cited in include/wvgpu.h).  Host slices are borrowed for the
// duration of the call only -- the library never retains a Go pointer -- and
// every status is a Go error carrying the library's thread-local message:
// each method pins its goroutine to one OS thread across the call and the
// wvg_last_error read (pin), and keeps its handles reachable until both are
// done, so a finalizer can never free a corpus a running call still uses.
// The binding is source only in this repository (no Go toolchain in the
// build image): build it with `go build -tags rocm` (INTEGRATION.md).
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../../../third_party/wvgpu/include
#cgo LDFLAGS: -L${SRCDIR}/../../../../../third_party/wvgpu/lib -lwvgpu -Wl,-rpath,$ORIGIN
#include <stdlib.h>
#include "wvgpu.h"
*/
import "C"

import (
	"fmt"
	"math"
	"runtime"
	"sync/atomic"
	"unsafe"

	"github.com/pkg/errors"
	"golang.org/x/sys/cpu"

	"github.com/weaviate/weaviate/adapters/repos/db/helpers"
)

// Corpus kinds and metrics (include/wvgpu.h); the metric names are the five
// Shard.initVectorIndex accepts (adapters/repos/db/shard.go:406-421).
const (
	KindF32 = int(C.WVG_KIND_F32)
	KindBQ  = int(C.WVG_KIND_BQ)
	KindPQ  = int(C.WVG_KIND_PQ)

	MetricL2        = int(C.WVG_METRIC_L2)
	MetricDot       = int(C.WVG_METRIC_DOT)
	MetricCosine    = int(C.WVG_METRIC_COSINE)
	MetricManhattan = int(C.WVG_METRIC_MANHATTAN)
	MetricHamming   = int(C.WVG_METRIC_HAMMING)
)

// MetricFromProvider maps distancer.Provider.Type() to the library's metric.
func MetricFromProvider(typ string) (int, error) {
	switch typ {
	case "l2-squared":
		return MetricL2, nil
	case "dot":
		return MetricDot, nil
	case "cosine-dot":
		return MetricCosine, nil
	case "manhattan":
		return MetricManhattan, nil
	case "hamming":
		return MetricHamming, nil
	}
	return 0, fmt.Errorf("wvgpu: unsupported distancer %q", typ)
}

// err maps a negative status to a Go error; the C side never aborts.
func err(rc C.int) error {
	if rc == C.WVG_OK {
		return nil
	}
	msg := C.GoString(C.wvg_last_error())
	if rc == C.WVG_ERR_DIM_MISMATCH {
		return errors.New(msg) // e.g. "insert called with a vector of the wrong size"
	}
	return fmt.Errorf("wvgpu %d: %s", int(rc), msg)
}

// pin locks the calling goroutine to its OS thread until the returned
// function runs (deferred by every method right at its start), so the C call
// and err()'s read of the library's thread-local wvg_last_error happen on the
// same thread -- the Go scheduler may otherwise move the goroutine between the
// two cgo calls -- and keeps the given handles reachable until then
// (runtime.KeepAlive), so no finalizer runs while a call uses them.
func pin(handles ...interface{}) func() {
	runtime.LockOSThread()
	return func() {
		runtime.UnlockOSThread()
		for _, h := range handles {
			runtime.KeepAlive(h)
		}
	}
}

func f32p(s []float32) *C.float {
	if len(s) == 0 {
		return nil
	}
	return (*C.float)(unsafe.Pointer(&s[0]))
}

func u64p(s []uint64) *C.uint64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&s[0]))
}

func u32p(s []uint32) *C.uint32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint32_t)(unsafe.Pointer(&s[0]))
}

func u8p(s []byte) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&s[0]))
}

// ABIVersion is the loaded library's ABI; CheckABI refuses a library built
// for another ABI than the header this package was compiled against (call it
// from the caller's package init); DeviceCount sizes WEAVIATE_GPU_DEVICES.
func ABIVersion() int { return int(C.wvg_abi_version()) }

func CheckABI() error {
	if got, want := ABIVersion(), int(C.WVG_ABI_VERSION); got != want {
		return fmt.Errorf("wvgpu: library ABI %d, binding built for ABI %d", got, want)
	}
	return nil
}

func DeviceCount() (int, error) {
	defer pin()()
	var n C.int
	if e := err(C.wvg_device_count(&n)); e != nil {
		return 0, e
	}
	return int(n), nil
}

// ---- context -----------------------------------------------------------------

// Ctx is one GPU's context.  It counts its open corpora: Close refuses while
// any is open, so no Corpus (nor its finalizer) ever uses a freed context.
type Ctx struct {
	h        *C.wvg_ctx
	corpora  int64
	borrowed bool // a device context of a Multi: closed by Multi.Close
}

func Open(device int) (*Ctx, error) {
	defer pin()()
	var h *C.wvg_ctx
	if e := err(C.wvg_open(C.int(device), &h)); e != nil {
		return nil, e
	}
	return &Ctx{h: h}, nil
}

// Options are fixed for the context's lifetime (wvg_options).  Start from
// DefaultOptions() and change what differs: OpenWith copies every field,
// including the three switches CacheReuse, BatchScreen and Coalesce, whose
// zero value turns the feature off.  OpenWith(dev, nil) = the defaults.
type Options struct {
	MFMAMinQueries uint32 // dot / cosine batches of at least this many queries use MFMA (default 32)
	CacheReuse     int32  // 1: consecutive scans reuse the Infinity Cache (default); 0: streaming
	MergeWaitUs    uint32 // query-stream merge wait bound (default 4 s)
	BatchScreen    int32  // 2: int8 screen (d 512/768/1024, else bf16) + exact rescore (default); 1: bf16; 0: exact only
	Coalesce       int32  // 1: concurrent single-query searches of a corpus share launches (default)
	HeapReplay     int32  // 1: BQ candidates / rescore exactly as Weaviate's heaps pick them (default)
}

func DefaultOptions() Options {
	var o C.wvg_options
	C.wvg_options_default(&o)
	return Options{uint32(o.mfma_min_queries), int32(o.cache_reuse), uint32(o.merge_wait_us), int32(o.batch_screen),
		int32(o.coalesce), int32(o.heap_replay)}
}

func OpenWith(device int, o *Options) (*Ctx, error) {
	defer pin()()
	var opt C.wvg_options
	C.wvg_options_default(&opt)
	if o != nil {
		opt.mfma_min_queries = C.uint32_t(o.MFMAMinQueries)
		opt.merge_wait_us = C.uint32_t(o.MergeWaitUs)
		opt.cache_reuse = C.int32_t(o.CacheReuse)
		opt.batch_screen = C.int32_t(o.BatchScreen)
		opt.coalesce = C.int32_t(o.Coalesce)
		opt.heap_replay = C.int32_t(o.HeapReplay)
	}
	var h *C.wvg_ctx
	if e := err(C.wvg_open_ex(C.int(device), &opt, &h)); e != nil {
		return nil, e
	}
	return &Ctx{h: h}, nil
}

// Close after every Corpus of the context is closed (an error otherwise).
func (c *Ctx) Close() error {
	defer pin(c)()
	if c.h == nil {
		return nil
	}
	if c.borrowed {
		return nil
	}
	if n := atomic.LoadInt64(&c.corpora); n != 0 {
		return fmt.Errorf("wvgpu: context still has %d open corpora", n)
	}
	e := err(C.wvg_close(c.h))
	c.h = nil
	return e
}

func (c *Ctx) Synchronize() error {
	defer pin(c)()
	return err(C.wvg_synchronize(c.h))
}

// MatchHostDistancer: on AMX + AVX-512 hosts Weaviate's init() picks l2_512 /
// dot_512 (D/l2_amd64.go:19-25, D/dot_product_amd64.go:19-25); the GPU then
// follows the same reduction order so distances stay bit-identical.
func (c *Ctx) MatchHostDistancer() error {
	defer pin(c)()
	order := C.WVG_ORDER_AVX256
	if cpu.X86.HasAVX512 && cpu.X86.HasAMXBF16 {
		order = C.WVG_ORDER_AVX512
	}
	return err(C.wvg_set_distance_order(c.h, C.int(order)))
}

// HostBuffer is page-locked memory for a reusable staging buffer (the R rows
// searchByVectorBQ gathers for its rescore, V/flat/index.go:375-385): copies
// from it skip the library's staging copy.  Free it with Free.
type HostBuffer struct {
	ctx *Ctx
	p   unsafe.Pointer
	n   uint64
}

func (c *Ctx) HostAlloc(bytes uint64) (*HostBuffer, error) {
	defer pin(c)()
	var p unsafe.Pointer
	if e := err(C.wvg_host_alloc(c.h, C.uint64_t(bytes), &p)); e != nil {
		return nil, e
	}
	return &HostBuffer{c, p, bytes}, nil
}

func (b *HostBuffer) Float32s() []float32 { return unsafe.Slice((*float32)(b.p), b.n/4) }

func (b *HostBuffer) Free() error {
	defer pin(b)()
	if b.p == nil {
		return nil
	}
	e := err(C.wvg_host_free(b.ctx.h, b.p))
	b.p = nil
	return e
}

// MeasureHBMRead: the device's streaming-read rate in GB/s (roofline ceiling).
func (c *Ctx) MeasureHBMRead(bytes uint64, reps uint32) (float64, error) {
	defer pin(c)()
	var gbps C.double
	if e := err(C.wvg_measure_hbm_read(c.h, C.uint64_t(bytes), C.uint32_t(reps), &gbps)); e != nil {
		return 0, e
	}
	return float64(gbps), nil
}

// ProfileStart / ProfileStop: per-dispatch scan-kernel time for the
// vector_index_durations_ms metric (usecases/monitoring/prometheus.go:292).
func (c *Ctx) ProfileStart() error {
	defer pin(c)()
	return err(C.wvg_profile_start(c.h))
}

func (c *Ctx) ProfileStop() (ms float64, launches uint64, e error) {
	defer pin(c)()
	var t C.double
	var n C.uint64_t
	e = err(C.wvg_profile_stop(c.h, &t, &n))
	return float64(t), uint64(n), e
}

// ---- device memory and streams (for the device-resident serving loop) ----------

// DeviceAlloc returns bytes of HBM on the context's GPU (zero-filled when zero:
// a search workspace must be).  Free it with DeviceFree once the work using it
// has finished (StreamSynchronize).
func (c *Ctx) DeviceAlloc(bytes uint64, zero bool) (unsafe.Pointer, error) {
	defer pin(c)()
	var p unsafe.Pointer
	z := C.int(0)
	if zero {
		z = 1
	}
	if e := err(C.wvg_device_alloc(c.h, C.uint64_t(bytes), z, &p)); e != nil {
		return nil, e
	}
	return p, nil
}

func (c *Ctx) DeviceFree(p unsafe.Pointer) error {
	defer pin(c)()
	return err(C.wvg_device_free(c.h, p))
}

// NewStream creates a non-blocking HIP stream for DeviceBuffers.Stream.
func (c *Ctx) NewStream() (unsafe.Pointer, error) {
	defer pin(c)()
	var s unsafe.Pointer
	if e := err(C.wvg_stream_create(c.h, &s)); e != nil {
		return nil, e
	}
	return s, nil
}

func (c *Ctx) StreamDestroy(s unsafe.Pointer) error {
	defer pin(c)()
	return err(C.wvg_stream_destroy(c.h, s))
}

func (c *Ctx) StreamSynchronize(s unsafe.Pointer) error {
	defer pin(c)()
	return err(C.wvg_stream_synchronize(c.h, s))
}

// CopyToDevice / CopyFromDevice copy between a Go slice and HBM on stream s;
// they return when the copy is done (the slice is not retained).
func (c *Ctx) CopyToDevice(dst unsafe.Pointer, src []float32, s unsafe.Pointer) error {
	defer pin(c)()
	return err(C.wvg_memcpy_h2d(c.h, dst, unsafe.Pointer(f32p(src)), C.uint64_t(4*len(src)), s))
}

func (c *Ctx) CopyFromDevice(dst []byte, src unsafe.Pointer, s unsafe.Pointer) error {
	defer pin(c)()
	return err(C.wvg_memcpy_d2h(c.h, unsafe.Pointer(u8p(dst)), src, C.uint64_t(len(dst)), s))
}

// ---- corpus --------------------------------------------------------------------

// Corpus is the device-resident copy of a flat index's rows (F32), its BQ
// cache or its PQ codes, indexed by docID: slot = id - idBase.
type Corpus struct {
	h    *C.wvg_corpus
	ctx  *Ctx
	kind int
	dims int
	pqM  int
}

func (c *Ctx) NewCorpus(kind, metric, dims int, idBase, capacity uint64) (*Corpus, error) {
	defer pin(c)()
	var h *C.wvg_corpus
	if e := err(C.wvg_corpus_create(c.h, C.int(kind), C.int(metric), C.uint32_t(dims), C.uint64_t(idBase),
		C.uint64_t(capacity), &h)); e != nil {
		return nil, e
	}
	x := &Corpus{h: h, ctx: c, kind: kind, dims: dims}
	atomic.AddInt64(&c.corpora, 1)
	// backstop for a leaked corpus (owners call Close): it runs only once x is
	// unreachable, i.e. after every method's pin has released it, and the
	// context cannot have been closed while x was open
	runtime.SetFinalizer(x, func(x *Corpus) { _ = x.Close() })
	return x, nil
}

// Close: flat.Drop / Shutdown.
func (x *Corpus) Close() error {
	defer pin(x)()
	if x.h == nil {
		return nil
	}
	e := err(C.wvg_corpus_destroy(x.h))
	x.h = nil
	atomic.AddInt64(&x.ctx.corpora, -1)
	runtime.SetFinalizer(x, nil)
	return e
}

// Reserve: cache.Grow (V/cache/sharded_lock_cache.go:251), contents kept.
func (x *Corpus) Reserve(capacity uint64) error {
	defer pin(x)()
	return err(C.wvg_corpus_reserve(x.h, C.uint64_t(capacity)))
}

func (x *Corpus) Info() (count, highWater, capacity uint64, e error) {
	defer pin(x)()
	var a, b, c C.uint64_t
	e = err(C.wvg_corpus_info(x.h, &a, &b, &c))
	return uint64(a), uint64(b), uint64(c), e
}

// Add: flat.Add / AddBatch (V/flat/index.go:247-274); flat is len(ids)*dims
// float32 (normalized inside for cosine, BQ / PQ encoded on the device).
func (x *Corpus) Add(ids []uint64, flat []float32) error {
	defer pin(x)()
	if len(ids) == 0 {
		return nil
	}
	if len(flat) != len(ids)*x.dims {
		return errors.New("insert called with a vector of the wrong size")
	}
	return err(C.wvg_corpus_upsert(x.h, u64p(ids), f32p(flat), C.uint64_t(len(ids)), C.uint32_t(x.dims)))
}

// AddCodes stores rows as the LSM holds them (F32 rows already normalized at
// Add, BQ uint64 words, PQ m bytes): restores, and the BQ / PQ caches.
func (x *Corpus) AddCodes(ids []uint64, codes unsafe.Pointer) error {
	defer pin(x)()
	if len(ids) == 0 {
		return nil
	}
	return err(C.wvg_corpus_upsert_codes(x.h, u64p(ids), codes, C.uint64_t(len(ids))))
}

// LoadKV: PostStartup bulk load straight from the LSM cursor's pairs
// (V/flat/index.go:640-681): keys 8-byte big-endian docIDs, values the rows.
func (x *Corpus) LoadKV(keys, values []byte, n int) error {
	defer pin(x)()
	if n == 0 {
		return nil
	}
	return err(C.wvg_corpus_load_kv(x.h, u8p(keys), u8p(values), C.uint64_t(n), C.uint64_t(len(values)/n)))
}

// Delete: flat.Delete (V/flat/index.go:276-295).
func (x *Corpus) Delete(ids ...uint64) error {
	defer pin(x)()
	if len(ids) == 0 {
		return nil
	}
	return err(C.wvg_corpus_delete(x.h, u64p(ids), C.uint64_t(len(ids))))
}

// Get: flat.vectorById (V/flat/index.go:401-407) of an F32 corpus.
func (x *Corpus) Get(id uint64) ([]float32, error) {
	defer pin(x)()
	out := make([]float32, x.dims)
	if e := err(C.wvg_corpus_get(x.h, C.uint64_t(id), unsafe.Pointer(&out[0]))); e != nil {
		return nil, e
	}
	return out, nil
}

// GetBatch: vectorById for many ids of an F32 corpus; ok[i] == false where
// ids[i] is not live.
func (x *Corpus) GetBatch(ids []uint64) ([]float32, []bool, error) {
	defer pin(x)()
	out := make([]float32, len(ids)*x.dims)
	ok := make([]uint8, len(ids))
	if len(ids) == 0 {
		return out, nil, nil
	}
	if e := err(C.wvg_corpus_get_batch(x.h, u64p(ids), C.uint64_t(len(ids)), unsafe.Pointer(&out[0]),
		u8p(ok))); e != nil {
		return nil, nil, e
	}
	return out, bools(ok), nil
}

// SetCodebook: the PQ encoders' centers [m][ks][dims/m] (CH/kmeans.go:85-93).
func (x *Corpus) SetCodebook(centers []float32, m, ks int) error {
	defer pin(x)()
	if e := err(C.wvg_pq_set_codebook(x.h, f32p(centers), C.uint32_t(m), C.uint32_t(ks))); e != nil {
		return e
	}
	x.pqM = m
	return nil
}

// EncodeFrom: the PQ preload of a resident float corpus (V/hnsw/compress.go:98-104).
func (x *Corpus) EncodeFrom(f32 *Corpus) error {
	defer pin(x, f32)()
	return err(C.wvg_pq_encode_corpus(x.h, f32.h))
}

func bools(b []uint8) []bool {
	out := make([]bool, len(b))
	for i, v := range b {
		out[i] = v != 0
	}
	return out
}

// ---- allow lists --------------------------------------------------------------------

// allowBitmap turns a helpers.AllowList into the ABI's bitmap over docIDs
// (bit i of word i/64).  nil means no filter.  A non-nil, empty list gives
// ok == false: the reference returns no results for it without scanning
// (V/flat/index.go:423-427), and so do the searches below -- passing nil to the
// library would instead search everything.
func allowBitmap(allow helpers.AllowList) (words []uint64, ok bool) {
	if allow == nil {
		return nil, true
	}
	if allow.IsEmpty() {
		return nil, false
	}
	words = make([]uint64, allow.Max()/64+1)
	it := allow.Iterator()
	for id, more := it.Next(); more; id, more = it.Next() {
		words[id/64] |= 1 << (id % 64)
	}
	return words, true
}

// ---- search ----------------------------------------------------------------------------

// Results of nq searches: [nq][k] ids / distances, Counts[q] valid entries.
type Results struct {
	K      int
	IDs    []uint64
	Dists  []float32
	Counts []uint32
}

// Query returns the valid part of query q's results.
func (r *Results) Query(q int) ([]uint64, []float32) {
	n := int(r.Counts[q])
	return r.IDs[q*r.K : q*r.K+n], r.Dists[q*r.K : q*r.K+n]
}

func emptyResults(nq, k int) *Results {
	r := &Results{K: k, IDs: make([]uint64, nq*k), Dists: make([]float32, nq*k), Counts: make([]uint32, nq)}
	for i := range r.IDs {
		r.IDs[i] = ^uint64(0) // no entry: id UINT64_MAX, distance +inf (as the library writes them)
		r.Dists[i] = float32(math.Inf(1))
	}
	return r
}

// Search: flat.SearchByVector (V/flat/index.go:307-334) for one query.
// Concurrent calls on one corpus (one per goroutine, as Weaviate's queries
// arrive) are coalesced inside the library into shared launches.
func (x *Corpus) Search(q []float32, k int, allow helpers.AllowList) ([]uint64, []float32, error) {
	r, e := x.SearchBatch(q, 1, k, allow)
	if e != nil {
		return nil, nil, e
	}
	ids, d := r.Query(0)
	return ids, d, nil
}

// SearchBatch: nq queries (qs is nq*dims floats) in one call.
func (x *Corpus) SearchBatch(qs []float32, nq, k int, allow helpers.AllowList) (*Results, error) {
	defer pin(x)()
	r := emptyResults(nq, k)
	if nq == 0 || k == 0 {
		return r, nil
	}
	if len(qs) != nq*x.dims {
		return nil, errors.New("vector lengths don't match")
	}
	words, ok := allowBitmap(allow)
	if !ok {
		return r, nil
	}
	if e := err(C.wvg_search(x.h, f32p(qs), C.uint32_t(nq), C.uint32_t(k), u64p(words), C.uint64_t(len(words)),
		u64p(r.IDs), f32p(r.Dists), u32p(r.Counts))); e != nil {
		return nil, e
	}
	return r, nil
}

// SearchBQRescore: flat.searchByVectorBQ (V/flat/index.go:347-389) with the
// float rows resident in f32 (same dims / idBase / metric as x).
func (x *Corpus) SearchBQRescore(f32 *Corpus, qs []float32, nq, k, rescoreLimit int,
	allow helpers.AllowList) (*Results, error) {
	defer pin(x, f32)()
	r := emptyResults(nq, k)
	if nq == 0 || k == 0 {
		return r, nil
	}
	words, ok := allowBitmap(allow)
	if !ok {
		return r, nil
	}
	if e := err(C.wvg_search_bq_rescore(x.h, f32.h, f32p(qs), C.uint32_t(nq), C.uint32_t(k),
		C.uint32_t(rescoreLimit), u64p(words), C.uint64_t(len(words)), u64p(r.IDs), f32p(r.Dists),
		u32p(r.Counts))); e != nil {
		return nil, e
	}
	return r, nil
}

// SearchBQCandidates: the first half of flat.searchByVectorBQ when the float
// rows stay in the LSM store (V/flat/index.go:355-374): the ids and Hamming
// distances findTopVectorsCached leaves in its heap of rescoreLimit, in the
// order heap.Pop() returns them.  Fetch those rows with vectorById and pass
// them, in this order, to Ctx.Rescore.
func (x *Corpus) SearchBQCandidates(qs []float32, nq, rescoreLimit int, allow helpers.AllowList) (*Results, error) {
	defer pin(x)()
	r := emptyResults(nq, rescoreLimit)
	if nq == 0 || rescoreLimit == 0 {
		return r, nil
	}
	words, ok := allowBitmap(allow)
	if !ok {
		return r, nil
	}
	if e := err(C.wvg_search_bq_candidates(x.h, f32p(qs), C.uint32_t(nq), C.uint32_t(rescoreLimit), u64p(words),
		C.uint64_t(len(words)), u64p(r.IDs), f32p(r.Dists), u32p(r.Counts))); e != nil {
		return nil, e
	}
	return r, nil
}

// SearchByDistance: the HNSW growing-limit loop's result (V/hnsw/search.go:
// 85-151) in one device pass; the buffer grows if the count exceeds it.
func (x *Corpus) SearchByDistance(q []float32, target float32, maxLimit int64,
	allow helpers.AllowList) ([]uint64, []float32, error) {
	defer pin(x)()
	words, ok := allowBitmap(allow)
	if !ok {
		return nil, nil, nil
	}
	capacity := 1024
	for {
		ids := make([]uint64, capacity)
		dists := make([]float32, capacity)
		var cnt C.uint64_t
		if e := err(C.wvg_search_by_distance(x.h, f32p(q), C.float(target), C.int64_t(maxLimit), u64p(words),
			C.uint64_t(len(words)), u64p(ids), f32p(dists), C.uint64_t(capacity), &cnt)); e != nil {
			return nil, nil, e
		}
		if int(cnt) <= capacity {
			return ids[:cnt], dists[:cnt], nil
		}
		capacity = int(cnt)
	}
}

// SearchByDistanceWindow: the flat index's own SearchByVectorDistance
// (V/flat/index.go:531-591 as written: one window of `window` results).
func (x *Corpus) SearchByDistanceWindow(q []float32, target float32, window int,
	allow helpers.AllowList) ([]uint64, []float32, error) {
	defer pin(x)()
	if window == 0 {
		return nil, nil, nil
	}
	words, ok := allowBitmap(allow)
	if !ok {
		return nil, nil, nil
	}
	ids := make([]uint64, window)
	dists := make([]float32, window)
	var cnt C.uint64_t
	if e := err(C.wvg_search_by_distance_window(x.h, f32p(q), C.float(target), C.uint32_t(window), u64p(words),
		C.uint64_t(len(words)), u64p(ids), f32p(dists), C.uint64_t(window), &cnt)); e != nil {
		return nil, nil, e
	}
	return ids[:cnt], dists[:cnt], nil
}

// DistanceByIDs: CompressorDistancer.DistanceToNode for a candidate batch
// (CH/compression.go:306-325; the HNSW rescore, V/hnsw/search.go:564-581).
func (x *Corpus) DistanceByIDs(q []float32, ids []uint64) ([]float32, []bool, error) {
	defer pin(x)()
	d := make([]float32, len(ids))
	ok := make([]uint8, len(ids))
	if len(ids) == 0 {
		return d, nil, nil
	}
	if e := err(C.wvg_corpus_distance_by_ids(x.h, f32p(q), u64p(ids), C.uint64_t(len(ids)), f32p(d),
		u8p(ok))); e != nil {
		return nil, nil, e
	}
	return d, bools(ok), nil
}

// DistanceByIDsBatch: the rescore step of many concurrent searches in one
// launch; qs is nq*dims floats, lists[q] query q's candidates.
func (x *Corpus) DistanceByIDsBatch(qs []float32, lists [][]uint64) ([][]float32, [][]bool, error) {
	defer pin(x)()
	nq := len(lists)
	if nq == 0 {
		return nil, nil, nil
	}
	off := make([]uint64, nq+1)
	for i, l := range lists {
		off[i+1] = off[i] + uint64(len(l))
	}
	ids := make([]uint64, 0, off[nq])
	for _, l := range lists {
		ids = append(ids, l...)
	}
	d := make([]float32, len(ids))
	ok := make([]uint8, len(ids))
	if e := err(C.wvg_corpus_distance_by_ids_batch(x.h, f32p(qs), C.uint32_t(nq), u64p(off), u64p(ids), f32p(d),
		u8p(ok))); e != nil {
		return nil, nil, e
	}
	ds, oks := make([][]float32, nq), make([][]bool, nq)
	for i := range lists {
		ds[i] = d[off[i]:off[i+1]]
		oks[i] = bools(ok[off[i]:off[i+1]])
	}
	return ds, oks, nil
}

// Rescore: the rescore loop of searchByVectorBQ (V/flat/index.go:375-385)
// over host rows fetched from the LSM (rows is len(ids)*dims floats; q
// normalized by the caller for cosine, as index.go:352 does).
func (c *Ctx) Rescore(metric int, q, rows []float32, ids []uint64, dims, k int) ([]uint64, []float32, error) {
	defer pin(c)()
	outIDs := make([]uint64, k)
	outD := make([]float32, k)
	if k == 0 || len(ids) == 0 {
		return nil, nil, nil
	}
	var cnt C.uint32_t
	if e := err(C.wvg_rescore(c.h, C.int(metric), f32p(q), f32p(rows), u64p(ids), C.uint64_t(len(ids)),
		C.uint32_t(dims), C.uint32_t(k), u64p(outIDs), f32p(outD), &cnt)); e != nil {
		return nil, nil, e
	}
	return outIDs[:cnt], outD[:cnt], nil
}

// ---- device-resident serving loop (queries and results in HBM) ------------------

// DeviceBuffers are HBM pointers owned by the caller (e.g. a serving loop's
// pools, from Ctx.DeviceAlloc); Stream is a Ctx.NewStream stream or nil.
type DeviceBuffers struct {
	Queries   unsafe.Pointer // float [nq][dims], normalized for cosine
	IDs       unsafe.Pointer // uint64 [nq][k]
	Dists     unsafe.Pointer // float [nq][k]
	Counts    unsafe.Pointer // uint32 [nq], may be nil
	Workspace unsafe.Pointer // WorkspaceSize bytes, zero-filled once
	WsBytes   uint64
	Stream    unsafe.Pointer
}

func (x *Corpus) WorkspaceSize(nq, k int) uint64 {
	defer pin(x)()
	return uint64(C.wvg_search_workspace_size(x.h, C.uint32_t(nq), C.uint32_t(k)))
}

// SearchDevice: nq searches on the device, asynchronous on b.Stream.
func (x *Corpus) SearchDevice(b DeviceBuffers, nq, k int) error {
	defer pin(x)()
	return err(C.wvg_search_device(x.h, (*C.float)(b.Queries), C.uint32_t(nq), C.uint32_t(k), (*C.uint64_t)(b.IDs),
		(*C.float)(b.Dists), (*C.uint32_t)(b.Counts), b.Workspace, C.size_t(b.WsBytes), b.Stream))
}

// SearchDevicePipelined: nq single-query scans in one query-stream launch.
func (x *Corpus) SearchDevicePipelined(b DeviceBuffers, nq, k int) error {
	defer pin(x)()
	return err(C.wvg_search_device_pipelined(x.h, (*C.float)(b.Queries), C.uint32_t(nq), C.uint32_t(k),
		(*C.uint64_t)(b.IDs), (*C.float)(b.Dists), (*C.uint32_t)(b.Counts), b.Workspace, C.size_t(b.WsBytes),
		b.Stream))
}

// CheckDevice surfaces a device-side failure of earlier device searches.
func (c *Ctx) CheckDevice(workspace, stream unsafe.Pointer) error {
	defer pin(c)()
	return err(C.wvg_search_device_check(c.h, workspace, stream))
}

// Multi-GPU shard merge (Index.objectVectorSearch, adapters/repos/db/index.go:
// 1644-1648): nlists packed blocks of PackedBytes(nq, kIn) bytes each.
func PackedBytes(nq, k int) uint64 { return uint64(C.wvg_topk_packed_bytes(C.uint32_t(nq), C.uint32_t(k))) }

func (c *Ctx) MergePacked(packed unsafe.Pointer, nq, nlists, kIn, k int, out DeviceBuffers) error {
	defer pin(c)()
	return err(C.wvg_topk_merge_packed(c.h, packed, C.uint32_t(nq), C.uint32_t(nlists), C.uint32_t(kIn),
		C.uint32_t(k), (*C.uint64_t)(out.IDs), (*C.float)(out.Dists), (*C.uint32_t)(out.Counts), out.Stream))
}

func (c *Ctx) MergeLists(dists, ids unsafe.Pointer, nq, nlists, kIn, k int, out DeviceBuffers) error {
	defer pin(c)()
	return err(C.wvg_topk_merge_device(c.h, (*C.float)(dists), (*C.uint64_t)(ids), C.uint32_t(nq),
		C.uint32_t(nlists), C.uint32_t(kIn), C.uint32_t(k), (*C.uint64_t)(out.IDs), (*C.float)(out.Dists),
		(*C.uint32_t)(out.Counts), out.Stream))
}

// ---- bulk primitives (distancer.Provider / compressionhelpers) --------------------

// BatchDist: Provider.SingleDist of q against n rows (D/provider.go:14-20).
func (c *Ctx) BatchDist(metric int, q, rows []float32, dims int) ([]float32, error) {
	defer pin(c)()
	n := len(rows) / dims
	out := make([]float32, n)
	if n == 0 {
		return out, nil
	}
	if e := err(C.wvg_distance_batch(c.h, C.int(metric), f32p(q), f32p(rows), C.uint64_t(n), C.uint32_t(dims),
		f32p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// Normalize: distancer.Normalize of n rows (D/normalize.go:16-32).
func (c *Ctx) Normalize(rows []float32, dims int) ([]float32, error) {
	defer pin(c)()
	out := make([]float32, len(rows))
	n := len(rows) / dims
	if n == 0 {
		return out, nil
	}
	if e := err(C.wvg_normalize_batch(c.h, f32p(rows), C.uint64_t(n), C.uint32_t(dims), f32p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// BQEncode: BinaryQuantizer.Encode (CH/binary_quantization.go:32-45).
func (c *Ctx) BQEncode(rows []float32, dims int) ([]uint64, error) {
	defer pin(c)()
	n := len(rows) / dims
	w := (dims + 63) / 64
	out := make([]uint64, n*w)
	if n == 0 {
		return out, nil
	}
	if e := err(C.wvg_bq_encode(c.h, f32p(rows), C.uint64_t(n), C.uint32_t(dims), u64p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// BQDistance: DistanceBetweenCompressedVectors of q against n codes (:47-56).
func (c *Ctx) BQDistance(q, codes []uint64) ([]float32, error) {
	defer pin(c)()
	w := len(q)
	if w == 0 {
		return nil, errors.New("empty code")
	}
	n := len(codes) / w
	out := make([]float32, n)
	if n == 0 {
		return out, nil
	}
	if e := err(C.wvg_bq_distance_batch(c.h, u64p(q), u64p(codes), C.uint64_t(n), C.uint32_t(w),
		f32p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// PQEncode: ProductQuantizer.Encode of host rows (CH/product_quantization.go:420-426).
func (c *Ctx) PQEncode(centers []float32, m, ks int, rows []float32, dims int) ([]byte, error) {
	defer pin(c)()
	n := len(rows) / dims
	out := make([]byte, n*m)
	if n == 0 {
		return out, nil
	}
	if e := err(C.wvg_pq_encode(c.h, f32p(centers), C.uint32_t(m), C.uint32_t(ks), f32p(rows), C.uint64_t(n),
		C.uint32_t(dims), u8p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// PQLUT: DistanceLookUpTable of one query (CH/product_quantization.go:62-104).
func (c *Ctx) PQLUT(metric int, centers []float32, m, ks, dims int, q []float32) ([]float32, error) {
	defer pin(c)()
	out := make([]float32, m*ks)
	if e := err(C.wvg_pq_lut(c.h, C.int(metric), f32p(centers), C.uint32_t(m), C.uint32_t(ks), C.uint32_t(dims),
		f32p(q), f32p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// PQADC: PQDistancer.Distance of n codes against a LUT (:352-361).
func (c *Ctx) PQADC(metric int, lut []float32, m, ks int, codes []byte) ([]float32, error) {
	defer pin(c)()
	n := len(codes) / m
	out := make([]float32, n)
	if n == 0 {
		return out, nil
	}
	if e := err(C.wvg_pq_adc_batch(c.h, C.int(metric), f32p(lut), C.uint32_t(m), C.uint32_t(ks), u8p(codes),
		C.uint64_t(n), f32p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// PQFit: ProductQuantizer.Fit (CH/product_quantization.go:372-418); centers
// [m][ks][dims/m] for SetCodebook.
func (c *Ctx) PQFit(data []float32, dims, m, ks int, trainingLimit, seed uint64) ([]float32, error) {
	defer pin(c)()
	n := len(data) / dims
	if n == 0 {
		return nil, errors.New("not enough data to fit kmeans")
	}
	centers := make([]float32, m*ks*(dims/m))
	if e := err(C.wvg_pq_fit(c.h, f32p(data), C.uint64_t(n), C.uint32_t(dims), C.uint32_t(m), C.uint32_t(ks),
		C.uint64_t(trainingLimit), C.uint64_t(seed), f32p(centers), nil)); e != nil {
		return nil, e
	}
	return centers, nil
}

// PQGlobalDistances: buildGlobalDistances (CH/product_quantization.go:236-251).
func (c *Ctx) PQGlobalDistances(metric int, centers []float32, m, ks, dims int) ([]float32, error) {
	defer pin(c)()
	out := make([]float32, m*ks*ks)
	if e := err(C.wvg_pq_global_distances(c.h, C.int(metric), f32p(centers), C.uint32_t(m), C.uint32_t(ks),
		C.uint32_t(dims), f32p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// PQSDC: DistanceBetweenCompressedVectors of code x against n codes (:297-311).
func (c *Ctx) PQSDC(metric int, table []float32, m, ks int, x, codes []byte) ([]float32, error) {
	defer pin(c)()
	n := len(codes) / m
	out := make([]float32, n)
	if n == 0 {
		return out, nil
	}
	if e := err(C.wvg_pq_sdc_batch(c.h, C.int(metric), f32p(table), C.uint32_t(m), C.uint32_t(ks), u8p(x),
		u8p(codes), C.uint64_t(n), f32p(out))); e != nil {
		return nil, e
	}
	return out, nil
}

// ---- several GPUs in one process ---------------------------------------------

// Multi serves one index from several GPUs of this process, as Weaviate's
// Index fans a search out over its shards (adapters/repos/db/index.go:
// 1567-1648): one context per device and, for distinct devices, one RCCL
// communicator per device inside the library.  Close refuses while a
// MultiCorpus of it is open.
type Multi struct {
	h       *C.wvg_multi
	corpora int64
}

// OpenMulti opens devices (e.g. every index of WEAVIATE_GPU_DEVICES) with
// options o (nil = defaults).
func OpenMulti(devices []int, o *Options) (*Multi, error) {
	defer pin()()
	if len(devices) == 0 {
		return nil, errors.New("wvgpu: OpenMulti needs at least one device")
	}
	devs := make([]C.int, len(devices))
	for i, d := range devices {
		devs[i] = C.int(d)
	}
	var opt C.wvg_options
	C.wvg_options_default(&opt)
	if o != nil {
		opt.mfma_min_queries = C.uint32_t(o.MFMAMinQueries)
		opt.merge_wait_us = C.uint32_t(o.MergeWaitUs)
		opt.cache_reuse = C.int32_t(o.CacheReuse)
		opt.batch_screen = C.int32_t(o.BatchScreen)
		opt.coalesce = C.int32_t(o.Coalesce)
		opt.heap_replay = C.int32_t(o.HeapReplay)
	}
	var h *C.wvg_multi
	if e := err(C.wvg_multi_open(&devs[0], C.int(len(devices)), &opt, &h)); e != nil {
		return nil, e
	}
	return &Multi{h: h}, nil
}

func (m *Multi) Close() error {
	defer pin(m)()
	if m.h == nil {
		return nil
	}
	if n := atomic.LoadInt64(&m.corpora); n != 0 {
		return fmt.Errorf("wvgpu: %d multi corpora still open", n)
	}
	e := err(C.wvg_multi_close(m.h))
	m.h = nil
	return e
}

// Info: the device count and whether the exchange runs over RCCL (false: peer
// copies, e.g. a one-GPU rehearsal with a repeated device).
func (m *Multi) Info() (ndev int, rccl bool, e error) {
	defer pin(m)()
	var n, r C.int
	e = err(C.wvg_multi_info(m.h, &n, &r))
	return int(n), r != 0, e
}

// MultiCorpus deals docIDs to the devices in contiguous slabs of rows/ndev
// (rounded up to 64): shard i holds [i*slab, (i+1)*slab).
type MultiCorpus struct {
	h     *C.wvg_multi_corpus
	m     *Multi
	dims  int
	shard int
}

func (m *Multi) NewCorpus(kind, metric, dims int, rows uint64) (*MultiCorpus, error) {
	defer pin(m)()
	var h *C.wvg_multi_corpus
	if e := err(C.wvg_multi_corpus_create(m.h, C.int(kind), C.int(metric), C.uint32_t(dims), C.uint64_t(rows),
		&h)); e != nil {
		return nil, e
	}
	atomic.AddInt64(&m.corpora, 1)
	x := &MultiCorpus{h: h, m: m, dims: dims}
	runtime.SetFinalizer(x, func(x *MultiCorpus) { _ = x.Close() })
	return x, nil
}

func (x *MultiCorpus) Close() error {
	defer pin(x)()
	if x.h == nil {
		return nil
	}
	e := err(C.wvg_multi_corpus_destroy(x.h))
	x.h = nil
	atomic.AddInt64(&x.m.corpora, -1)
	runtime.SetFinalizer(x, nil)
	return e
}

// Shard i's slab: its docID base and rows (its own corpus handle stays
// inside the library; per-shard work goes through the Multi methods).
func (x *MultiCorpus) Shard(i int) (idBase, slabRows uint64, e error) {
	defer pin(x)()
	var b, s C.uint64_t
	e = err(C.wvg_multi_corpus_shard(x.h, C.int(i), nil, &b, &s))
	return uint64(b), uint64(s), e
}

// Add / AddBatch / Delete routed to the shard owning each docID.
func (x *MultiCorpus) AddBatch(ids []uint64, vectors [][]float32) error {
	defer pin(x)()
	if len(ids) != len(vectors) {
		return errors.Errorf("ids and vectors have different lengths")
	}
	if len(ids) == 0 {
		return nil
	}
	flat := make([]float32, 0, len(ids)*x.dims)
	for _, v := range vectors {
		if len(v) != x.dims {
			return errors.Errorf("insert called with a vector of the wrong size")
		}
		flat = append(flat, v...)
	}
	return err(C.wvg_multi_corpus_upsert(x.h, u64p(ids), f32p(flat), C.uint64_t(len(ids)), C.uint32_t(x.dims)))
}

func (x *MultiCorpus) Delete(ids ...uint64) error {
	defer pin(x)()
	return err(C.wvg_multi_corpus_delete(x.h, u64p(ids), C.uint64_t(len(ids))))
}

// SetCodebook: the PQ codebook (centers [m][ks][dims/m]) of every shard.
func (x *MultiCorpus) SetCodebook(centers []float32, m, ks int) error {
	defer pin(x)()
	return err(C.wvg_multi_corpus_set_codebook(x.h, f32p(centers), C.uint32_t(m), C.uint32_t(ks)))
}

// SearchBatch: nq queries over every shard -- the per-device scans, one RCCL
// all-gather of their top-k blocks, the merge (index.go:1644-1648).
func (x *MultiCorpus) SearchBatch(qs []float32, nq, k int, allow helpers.AllowList) (*Results, error) {
	defer pin(x)()
	r := emptyResults(nq, k)
	if nq == 0 || k == 0 {
		return r, nil
	}
	words, ok := allowBitmap(allow)
	if !ok {
		return r, nil
	}
	if e := err(C.wvg_multi_search(x.h, f32p(qs), C.uint32_t(nq), C.uint32_t(k), u64p(words),
		C.uint64_t(len(words)), u64p(r.IDs), f32p(r.Dists), u32p(r.Counts))); e != nil {
		return nil, e
	}
	return r, nil
}

// Ctx: device i's context (for that device's own corpora and bulk calls);
// owned by the Multi, so its Close does nothing.
func (m *Multi) Ctx(i int) (*Ctx, error) {
	defer pin(m)()
	var h *C.wvg_ctx
	if e := err(C.wvg_multi_ctx(m.h, C.int(i), &h)); e != nil {
		return nil, e
	}
	return &Ctx{h: h, borrowed: true}, nil
}
