// Row f4: the data half of sstable.CheckIntegrity
// (/root/reference/lsm/sstable/sstable.go:2287-2420) through libhundcrc:
// md5.Sum of every record (:2362) as one GPU batch, NewMerkleTree(hashes,
// true) (merkle_tree.go:38-87) as level arrays, and
// Validate(Deserialize(stored)) (:124-153, :219-250).  The pointer tree of
// merkle_tree.go stays for everything else (flush-time construction,
// Serialize for persistence); this file only adds the batch path.
// Not compiled here (no Go toolchain); see INTEGRATION.md.
package merkle_tree

/*
#cgo CFLAGS: -I${SRCDIR}/../../../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../../../hunddb_amd -lhundcrc
#include <stdlib.h>
#include "hundcrc.h"
*/
import "C"

import (
	"fmt"
	"unsafe"
)

func u8p(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// RecordHashes returns md5.Sum(data[off[i]:off[i]+lens[i]]) for every record
// (sstable.go:2362), computed in one GPU batch.  Panics without a GPU (no
// silent CPU fallback), like the other batched entries of utils/crc.
func RecordHashes(data []byte, off []uint64, lens []uint32) [][16]byte {
	out := make([][16]byte, len(off))
	if len(off) == 0 {
		return out
	}
	rc := C.hc_md5_messages(u8p(data), (*C.uint64_t)(unsafe.Pointer(&off[0])),
		(*C.uint32_t)(unsafe.Pointer(&lens[0])), C.uint64_t(len(off)), (*C.uint8_t)(unsafe.Pointer(&out[0][0])))
	if rc != C.HC_OK {
		panic(fmt.Sprintf("hc_md5_messages: %s", C.GoString(C.hc_strerror(rc))))
	}
	return out
}

// CheckRecords is CheckIntegrity's steps 2-4 over records already read (and
// CRC-verified) from the data component: the tree over their hashes (an
// empty component hashes as md5.Sum([]byte{}), :2368-2371) validated against
// the stored serialization.  It returns whether the roots agree and, when
// they do not, the built-tree leaf hash DeepValidate reports (at most one:
// Deserialize builds a left chain), which the caller maps back to a block
// through hashToOffset (:2413).  Go panics on a nil stored root; this
// returns an error instead.
func CheckRecords(data []byte, off []uint64, lens []uint32, stored []byte) (bool, [][16]byte, error) {
	leaves := RecordHashes(data, off, lens)
	n := len(leaves)
	levels := make([]byte, 16*int(C.hc_merkle_nodes(C.uint64_t(n))))
	var src *C.uint8_t
	if n > 0 {
		src = (*C.uint8_t)(unsafe.Pointer(&leaves[0][0]))
	}
	if rc := C.hc_merkle_levels(src, C.uint64_t(n), u8p(levels)); rc != C.HC_OK {
		return false, nil, fmt.Errorf("failed to create Merkle tree: %s", C.GoString(C.hc_strerror(rc)))
	}
	var valid C.int
	var nm C.uint64_t
	var mismBuilt, mismStored [16]byte
	rc := C.hc_merkle_validate(u8p(levels), C.uint64_t(n), u8p(stored), C.uint64_t(len(stored)), &valid,
		(*C.uint8_t)(unsafe.Pointer(&mismBuilt[0])), (*C.uint8_t)(unsafe.Pointer(&mismStored[0])), &nm)
	if rc != C.HC_OK {
		return false, nil, fmt.Errorf("failed to validate Merkle tree: %s", C.GoString(C.hc_strerror(rc)))
	}
	if valid != 0 {
		return true, nil, nil
	}
	if nm == 0 {
		return false, nil, nil
	}
	return false, [][16]byte{mismBuilt}, nil
}
