// Package crc is the cgo binding of HundDB's utils/crc onto libhundcrc.so
// (include/hundcrc.h): a drop-in for /root/reference/utils/crc/crc_util.go
// with the identical exported surface (names, types, constant kinds, error
// texts), so lsm/wal, lsm/block_manager, lsm/sstable, lsm and probabilistic/*
// compile and behave unchanged.  Not compiled in this repository (no Go
// toolchain here or on the GPU box); see INTEGRATION.md.
package crc

/*
#cgo CFLAGS: -I${SRCDIR}/../../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../../hunddb_amd -lhundcrc -Wl,-rpath,${SRCDIR}/../../../../hunddb_amd
#include <stdint.h>
#include "hundcrc.h"
*/
import "C"

import (
	"errors"
	"sync"
	"unsafe"
)

// GPUAvailable reports whether a gfx950 device is visible, probed on the first
// call only (importing the package starts no HIP runtime).  The utils/crc
// drop-ins work without one (single buffers and AddCRCsToData run on the host
// CPU then); the batched helpers below (CheckBlocksIntegrity, AddCRCToBlocks,
// ReadVerified*) return an error instead, never a silent CPU fallback.  A
// deployment that relies on them should call GPUAvailable at startup rather
// than discover it mid-flush.
func GPUAvailable() bool {
	gpuOnce.Do(func() { gpuAvail = C.hc_device_count() > 0 })
	return gpuAvail
}

var (
	gpuOnce  sync.Once
	gpuAvail bool
)

// BLOCK_SIZE keeps the typed-uint64 form and CRC_SIZE the untyped form of
// crc_util.go:11-12 (CRC_SIZE is used in both int and uint64 contexts).
const BLOCK_SIZE = 1024 * uint64(4)
const CRC_SIZE = 4

func ptr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

func goErr(rc C.int) error {
	if rc == C.HC_OK {
		return nil
	}
	// < 0: a library failure (no GPU for a batch, HIP error) -- an error value,
	// never a silent fallback; >= 1: the exact crc_util.go texts
	return errors.New(C.GoString(C.hc_strerror(rc)))
}

// GetCRC calculates CRC32 checksum over a byte array (crc_util.go:15).
func GetCRC(data []byte) uint32 {
	return uint32(C.hc_crc32_ieee(ptr(data), C.size_t(len(data))))
}

// AddCRCToBlockData stamps data[0:4] in place and returns data (crc_util.go:21).
func AddCRCToBlockData(data []byte) []byte {
	if len(data) < CRC_SIZE {
		return data
	}
	// cannot fail on the host path; only HC_FORCE_GPU (test mode) reaches the GPU
	if err := goErr(C.hc_add_crc_block(ptr(data), C.size_t(len(data)))); err != nil {
		panic("hundcrc: AddCRCToBlockData: " + err.Error())
	}
	return data
}

// AddCRCsToData frames data into BLOCK_SIZE blocks with a CRC each (crc_util.go:41).
// Inputs above the library's GPU threshold are CRC'd in one GPU batch; when
// that batch cannot run or fails (no gfx950, a device or pinned allocation
// failure, a HIP runtime error) the library finishes the CRCs on the host path
// and counts the event (hc_stats), so this cannot fail, as the reference
// cannot.  hc_add_crcs returns ^0 only for a dst smaller than
// hc_add_crcs_size(n), which the make() below rules out, or under the
// HC_FORCE_GPU test mode; the panic is kept for those.
func AddCRCsToData(serializedData []byte) []byte {
	out := make([]byte, int(C.hc_add_crcs_size(C.size_t(len(serializedData)))))
	if len(out) == 0 {
		return out
	}
	w := C.hc_add_crcs(ptr(serializedData), C.size_t(len(serializedData)), ptr(out), C.size_t(len(out)))
	if w == ^C.size_t(0) {
		panic("hundcrc: AddCRCsToData: output buffer too small (or HC_FORCE_GPU batch failed)")
	}
	return out
}

// SizeAfterAddingCRCs (crc_util.go:69).
func SizeAfterAddingCRCs(originalSize uint64) uint64 {
	return uint64(C.hc_size_after_crcs(C.uint64_t(originalSize)))
}

// SizeWithoutCRCs (crc_util.go:79).
func SizeWithoutCRCs(originalSize uint64) uint64 {
	return uint64(C.hc_size_without_crcs(C.uint64_t(originalSize)))
}

// CheckBlockIntegrity (crc_util.go:88): nil, "invalid block data" or "CRC mismatch in block".
func CheckBlockIntegrity(blockData []byte) error {
	return goErr(C.hc_check_block(ptr(blockData), C.size_t(len(blockData))))
}

// FixLastBlockCRC (crc_util.go:106): restamps the last complete block in place.
func FixLastBlockCRC(data []byte) error {
	return goErr(C.hc_fix_last_block(ptr(data), C.size_t(len(data))))
}

// ---- batched entries (new; the GPU hot path) ------------------------------

// gpuBatchMinBlocks is where one GPU batch beats the per-block host loop for
// a single caller on pageable (Go) memory: 1024 blocks of 4 KiB
// (tools/crossover.py; DESIGN.md 5.2).  Below it the batched helpers run the
// reference's own loop on the host path of the library.
const gpuBatchMinBlocks = 1024

// CheckBlocksIntegrity verifies every blockSize-byte block of data (the
// per-block loop of BlockManager.ReadFromDisk, block_manager.go:203-235, and
// WAL recovery, wal.go:366-403): one GPU batch from gpuBatchMinBlocks blocks,
// CheckBlockIntegrity per block below.  It returns the index of the first
// failing block (-1 if none) and that block's error.
func CheckBlocksIntegrity(data []byte, blockSize int) (int, error) {
	n := len(data) / blockSize
	if n < gpuBatchMinBlocks {
		for i := 0; i < n; i++ {
			if err := CheckBlockIntegrity(data[i*blockSize : (i+1)*blockSize]); err != nil {
				return i, err
			}
		}
		return -1, nil
	}
	var first C.int64_t = -1
	rc := C.hc_verify_blocks(ptr(data), nil, nil, C.uint64_t(blockSize), C.uint32_t(blockSize),
		C.uint64_t(n), nil, &first)
	return int(first), goErr(rc)
}

// AddCRCToBlocks stamps every blockSize-byte block of data (flushBlock over a
// run of WAL blocks, wal.go:260-271): one GPU batch from gpuBatchMinBlocks
// blocks, AddCRCToBlockData per block below.
func AddCRCToBlocks(data []byte, blockSize int) error {
	n := len(data) / blockSize
	if n < gpuBatchMinBlocks {
		for i := 0; i < n; i++ {
			AddCRCToBlockData(data[i*blockSize : (i+1)*blockSize])
		}
		return nil
	}
	return goErr(C.hc_stamp_blocks(ptr(data), nil, nil, C.uint64_t(blockSize), C.uint32_t(blockSize), C.uint64_t(n)))
}

// CheckBlocksIntegrityOn is CheckBlocksIntegrity over several GPUs of this
// process: the blocks are split into contiguous ranges (hc_shard_plan), range d
// is verified on devices[d] through its own host pipeline, so every GPU's PCIe
// link carries its share.  Same result as CheckBlocksIntegrity.
func CheckBlocksIntegrityOn(data []byte, blockSize int, devices []int) (int, error) {
	n := len(data) / blockSize
	devs := make([]C.int, len(devices))
	for i, d := range devices {
		devs[i] = C.int(d)
	}
	if len(devs) == 0 {
		return CheckBlocksIntegrity(data, blockSize)
	}
	var first C.int64_t = -1
	rc := C.hc_multi_verify_blocks(ptr(data), nil, nil, C.uint64_t(blockSize), C.uint32_t(blockSize),
		C.uint64_t(n), nil, &first, C.int(len(devs)), &devs[0], nil)
	return int(first), goErr(rc)
}

// AddCRCToBlocksOn is AddCRCToBlocks over several GPUs (see CheckBlocksIntegrityOn).
func AddCRCToBlocksOn(data []byte, blockSize int, devices []int) error {
	n := len(data) / blockSize
	devs := make([]C.int, len(devices))
	for i, d := range devices {
		devs[i] = C.int(d)
	}
	if len(devs) == 0 {
		return AddCRCToBlocks(data, blockSize)
	}
	return goErr(C.hc_multi_stamp_blocks(ptr(data), nil, nil, C.uint64_t(blockSize), C.uint32_t(blockSize),
		C.uint64_t(n), C.int(len(devs)), &devs[0], nil))
}

// ReadVerified is BlockManager.ReadFromDisk (block_manager.go:189-242) minus
// the file I/O: raw holds the blocks from startOffset/blockSize on, as read
// (cache or disk).  Every touched block is verified in one batch, then the
// payload bytes and the final physical offset are returned exactly as the Go
// loop returns them; on a bad block it returns that block's error.
func ReadVerified(raw []byte, blockSize uint16, startOffset, size uint64) ([]byte, uint64, error) {
	out := make([]byte, size)
	var final C.uint64_t
	var bad C.int64_t
	rc := C.hc_read_from_disk(ptr(raw), C.uint64_t(len(raw)), C.uint32_t(blockSize),
		C.uint64_t(startOffset), C.uint64_t(size), ptr(out), &final, &bad)
	if err := goErr(rc); err != nil {
		return nil, 0, err
	}
	return out, uint64(final), nil
}

// ReadBlocksTouched is the number of blocks ReadFromDisk(startOffset, size)
// touches (block_manager.go:191-235): the length of ReadVerifiedCached's masks.
func ReadBlocksTouched(blockSize uint16, startOffset, size uint64) int {
	return int(C.hc_read_blocks_touched(C.uint32_t(blockSize), C.uint64_t(startOffset), C.uint64_t(size)))
}

// ReadVerifiedCached is ReadVerified with the block cache's verified bits
// (row f1): verified[i] == true marks block i of raw (relative to
// startOffset/blockSize) as already checked -- a cache entry whose bytes were
// CRC-checked (on an earlier read, or when WriteBlock cached its copy) and that
// no caller can have changed since -- so it is not hashed again.
// On return verified[i] is also true for every block this call verified clean,
// which the caller records in its cache entries.
func ReadVerifiedCached(raw []byte, blockSize uint16, startOffset, size uint64, verified []bool) ([]byte, uint64, error) {
	k := ReadBlocksTouched(blockSize, startOffset, size)
	bits := make([]uint32, (k+31)/32)
	for i := 0; i < k && i < len(verified); i++ {
		if verified[i] {
			bits[i>>5] |= 1 << uint(i&31)
		}
	}
	out := make([]byte, size)
	var final C.uint64_t
	var bad C.int64_t
	var bitsPtr *C.uint32_t
	if len(bits) > 0 {
		bitsPtr = (*C.uint32_t)(unsafe.Pointer(&bits[0]))
	}
	rc := C.hc_read_from_disk_v(ptr(raw), C.uint64_t(len(raw)), C.uint32_t(blockSize), C.uint64_t(startOffset),
		C.uint64_t(size), bitsPtr, ptr(out), &final, &bad, nil)
	for i := 0; i < k && i < len(verified); i++ {
		verified[i] = bits[i>>5]>>uint(i&31)&1 == 1
	}
	if err := goErr(rc); err != nil {
		return nil, 0, err
	}
	return out, uint64(final), nil
}

// WalWindow is what WalReplay returns for one window of WAL blocks.
type WalWindow struct {
	Records    [][]byte // serialized records (what record.Deserialize receives), in order
	EndBlocks  []uint64 // block (index within the window) in which each record completes
	PendBlock  int64    // where the fragments pending at the window's end start (-1: none)
	PendOffset uint64
	StopBlock  uint64 // after an error: the failing block (index within the window) ...
	StopOffset uint64 // ... and the offset wal.go's position would hold there
}

// WalReplay is one window of WAL recovery (row f3; wal.go:362-455 minus the
// file I/O and the memtable): blocks holds written WAL blocks of blockSize
// bytes back to back, parsing starts at startOffset of the first block.  Every
// block is verified in one batch (GPU from 1024 blocks, DESIGN.md 5.2), then FULL payloads and
// reassembled FIRST/MIDDLE/LAST fragments come back in order as slices of one
// buffer.  A bad block ("CRC mismatch in block") or a framing error ("unknown
// fragment type", or a header/payload past its block where Go panics) returns
// the records before it with the error and StopBlock/StopOffset.
func WalReplay(blocks []byte, blockSize int, startOffset uint64) (WalWindow, error) {
	nb := len(blocks) / blockSize
	slots := nb*((blockSize-CRC_SIZE)/17+1) + 1
	buf := make([]byte, len(blocks)+1)
	off := make([]uint64, slots)
	ln := make([]uint64, slots)
	endBlk := make([]uint64, slots)
	pend := make([]uint64, 2)
	var nrec, posBlock, posOffset C.uint64_t
	var bad C.int64_t = -1
	rc := C.hc_wal_replay_v(ptr(blocks), C.uint64_t(nb), C.uint32_t(blockSize), 0, C.uint64_t(startOffset), 0,
		ptr(buf), C.uint64_t(len(buf)), (*C.uint64_t)(unsafe.Pointer(&off[0])), (*C.uint64_t)(unsafe.Pointer(&ln[0])),
		(*C.uint64_t)(unsafe.Pointer(&endBlk[0])), C.uint64_t(slots), &nrec, &posBlock, &posOffset, &bad,
		(*C.uint64_t)(unsafe.Pointer(&pend[0])))
	w := WalWindow{PendBlock: -1, StopBlock: uint64(posBlock), StopOffset: uint64(posOffset)}
	if rc < 0 {
		return w, goErr(rc)
	}
	w.Records = make([][]byte, int(nrec))
	for i := range w.Records {
		w.Records[i] = buf[off[i] : off[i]+ln[i] : off[i]+ln[i]]
	}
	w.EndBlocks = endBlk[:int(nrec)]
	if pend[0] != ^uint64(0) {
		w.PendBlock, w.PendOffset = int64(pend[0]), pend[1]
	}
	return w, goErr(rc)
}

// LibraryStats are the library's process-wide event counters (hc_stats): how
// many AddCRCsToData / ReadFromDisk / WAL-recovery batches ran on the GPU, and
// how many finished on the host path because no gfx950 was usable or the GPU
// batch failed (LastFallbackError: the last failure's library code).  For
// metrics; the reference has no counterpart.
type LibraryStats struct {
	AddCRCsGPU, AddCRCsHostSmall, AddCRCsHostNoDev, AddCRCsGPUFallback uint64
	LastFallbackError                                                  int64
	ReadGPU, ReadGPUFallback, WALGPU, WALGPUFallback, NoDevHost        uint64
}

// Stats reads the counters.
func Stats() LibraryStats {
	var out C.hc_stats_t
	C.hc_stats(&out)
	return LibraryStats{
		AddCRCsGPU: uint64(out.add_crcs_gpu), AddCRCsHostSmall: uint64(out.add_crcs_host_small),
		AddCRCsHostNoDev: uint64(out.add_crcs_host_nodev), AddCRCsGPUFallback: uint64(out.add_crcs_gpu_fallback),
		LastFallbackError: int64(out.last_fallback_error),
		ReadGPU: uint64(out.read_gpu), ReadGPUFallback: uint64(out.read_gpu_fallback),
		WALGPU: uint64(out.wal_gpu), WALGPUFallback: uint64(out.wal_gpu_fallback), NoDevHost: uint64(out.nodev_host),
	}
}
