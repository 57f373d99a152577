// Row f1 of SURVEY.md section 8: BlockManager.ReadFromDisk with ONE batched
// verify per call and a verified bit per cached block, so cache hits are not
// re-verified (the CRC amplification of /root/reference/lsm/block_manager/
// block_manager.go:72-77 + :215, where every ReadFromDisk re-hashes blocks the
// LRU cache returned).  The maintainer's patch to lsm/block_manager: the cache
// value becomes *cachedBlock, ReadBlock/WriteBlock fill it, and ReadFromDisk
// collects the touched blocks and verifies them through
// crc_util.ReadVerifiedCached.  Not compiled in this repository (no Go
// toolchain here or on the GPU box); INTEGRATION.md section 3 explains it.
package block_manager

import (
	"errors"
	lru_cache "hunddb/lsm/lru_cache"
	block_location "hunddb/model/block_location"
	crc_util "hunddb/utils/crc"
	"sync"
	"sync/atomic"
)

// cachedBlock is what the block cache holds: the block's bytes and whether
// their CRC has been checked.  Blocks the engine writes carry a valid CRC by
// construction (AddCRCsToData / AddCRCToBlockData before WriteBlock), so
// WriteBlock caches them as verified; blocks read from disk start unverified.
type cachedBlock struct {
	data     []byte
	verified atomic.Bool
}

// BlockManager as in block_manager.go:34-38 with the cache value changed.
type BlockManager struct {
	blockSize   uint16
	blockCache  *lru_cache.LRUCache[block_location.BlockLocation, *cachedBlock]
	fileMutexes sync.Map
}

// readCached replaces ReadBlock (block_manager.go:72-98) on the read path: the
// same cache / file-lock / double-check protocol, returning the cache entry.
func (bm *BlockManager) readCached(location block_location.BlockLocation) (*cachedBlock, error) {
	if cb, err := bm.blockCache.Get(location); err == nil {
		return cb, nil
	}
	mutex := bm.getFileMutex(location.FilePath)
	mutex.RLock()
	defer mutex.RUnlock()
	if cb, err := bm.blockCache.Get(location); err == nil {
		return cb, nil
	}
	block, err := bm.readBlockFromDisk(location)
	if err != nil {
		return nil, errors.New("block not read successfully")
	}
	cb := &cachedBlock{data: block}
	bm.blockCache.Put(location, cb)
	return cb, nil
}

// ReadBlock keeps its signature (block_manager.go:72): the bytes only.
func (bm *BlockManager) ReadBlock(location block_location.BlockLocation) ([]byte, error) {
	cb, err := bm.readCached(location)
	if err != nil {
		return nil, err
	}
	return cb.data, nil
}

// WriteBlock as block_manager.go:101-114; the written block is cached as verified.
func (bm *BlockManager) WriteBlock(location block_location.BlockLocation, data []byte) error {
	mutex := bm.getFileMutex(location.FilePath)
	mutex.Lock()
	defer mutex.Unlock()
	if err := bm.writeBlockToDisk(location, data); err != nil {
		return errors.New("block not written successfully")
	}
	cb := &cachedBlock{data: data}
	cb.verified.Store(true)
	bm.blockCache.Put(location, cb)
	return nil
}

// ReadFromDisk (block_manager.go:189-242): same arguments, results and error
// values; every touched block not yet verified is checked in one batch (GPU from
// 256 blocks), cached blocks already verified are not hashed again, and blocks
// verified here are marked in the cache.
func (bm *BlockManager) ReadFromDisk(filePath string, startOffset uint64, size uint64) ([]byte, uint64, error) {
	bs := uint64(bm.blockSize)
	k := crc_util.ReadBlocksTouched(bm.blockSize, startOffset, size)
	first := startOffset / bs
	raw := make([]byte, 0, uint64(k)*bs)
	entries := make([]*cachedBlock, k)
	verified := make([]bool, k)
	for i := 0; i < k; i++ {
		cb, err := bm.readCached(block_location.BlockLocation{FilePath: filePath, BlockIndex: first + uint64(i)})
		if err != nil {
			return nil, 0, err // the Go loop fails at the first unreadable block too
		}
		entries[i] = cb
		verified[i] = cb.verified.Load()
		raw = append(raw, cb.data...)
	}
	out, final, err := crc_util.ReadVerifiedCached(raw, bm.blockSize, startOffset, size, verified)
	for i, v := range verified {
		if v {
			entries[i].verified.Store(true)
		}
	}
	if err != nil {
		return nil, 0, err
	}
	return out, final, nil
}
