// Row f3 of SURVEY.md section 8: WAL recovery with one batched verify and a
// parallel parse per window of blocks, instead of one ReadBlock +
// CheckBlockIntegrity + processBlockForRecovery per block
// (/root/reference/lsm/wal/wal.go:362-455).  The maintainer's patch to
// lsm/wal: recoverMemtable below replaces wal.go:362-406, and
// processBlockForRecovery (:411-455) is no longer called; the block reads
// still go through the block manager (its cache and file locks).  Not compiled
// in this repository (no Go toolchain here or on the GPU box); INTEGRATION.md
// section 3 explains it.
package wal

import (
	"fmt"
	bm "hunddb/lsm/block_manager"
	memtable "hunddb/lsm/memtable"
	block_location "hunddb/model/block_location"
	record "hunddb/model/record"
	crc "hunddb/utils/crc"
)

// recoverWindowBlocks is how many blocks one replay call takes (16 MiB of
// 4 KiB blocks: one GPU verify batch, one parallel parse); a record whose
// fragments span more than a window widens it.
const recoverWindowBlocks = 4096

type walBlock struct{ log, block uint64 }

// recoverMemtable (wal.go:362-406) replays records from position into the
// memtable until it is full or the WAL ends, with the reference's position
// and error behaviour:
//   - memtable.IsFull after a Put: the next memtable starts at the block
//     after the one that record completed in (wal.go:392-397);
//   - a block that cannot be read, or fails its CRC: the records completed
//     before it are Put, then the error is returned with position on it;
//   - the WAL's end: position moves past the last log (wal.go:400-405), and
//     fragments still pending there are dropped, as Go's fragmentBuffer is.
func (wal *WAL) recoverMemtable(mt *memtable.MemTable, position *WalPosition) error {
	if position.LogIndex > wal.lastLogIndex {
		return nil
	}
	blockManager := bm.GetBlockManager()
	// the written blocks from position on, every log in order (wal.go:365-372)
	var locs []walBlock
	for li := position.LogIndex; li <= wal.lastLogIndex; li++ {
		end := wal.logSize
		if li == wal.lastLogIndex {
			end = wal.blocksWrittenInLastLog
		}
		b := uint64(0)
		if li == position.LogIndex {
			b = position.BlockIndex
		}
		for ; b < end; b++ {
			locs = append(locs, walBlock{li, b})
		}
	}
	path := func(l walBlock) string { return fmt.Sprintf("%s/wal_%d.log", wal.logsPath, l.log) }
	setPos := func(k int, off uint64) {
		position.LogIndex, position.BlockIndex, position.Offset = locs[k].log, locs[k].block, off
	}

	start, offset, window := 0, position.Offset, recoverWindowBlocks
	for start < len(locs) {
		hi := start + window
		if hi > len(locs) {
			hi = len(locs)
		}
		raw := make([]byte, 0, (hi-start)*int(BLOCK_SIZE))
		var readErr error
		readAt := hi
		for k := start; k < hi; k++ {
			block, err := blockManager.ReadBlock(block_location.BlockLocation{FilePath: path(locs[k]), BlockIndex: locs[k].block})
			if err != nil {
				readErr = fmt.Errorf("failed to read block %s:%d: %w", path(locs[k]), locs[k].block, err)
				readAt = k
				break
			}
			raw = append(raw, block...)
		}
		w, err := crc.WalReplay(raw, int(BLOCK_SIZE), offset)
		for i, payload := range w.Records {
			mt.Put(record.Deserialize(payload))
			if mt.IsFull() { // wal.go:392-397
				setPos(start+int(w.EndBlocks[i]), crc.CRC_SIZE)
				position.BlockIndex++
				return nil
			}
		}
		if err != nil {
			k := start + int(w.StopBlock)
			setPos(k, w.StopOffset)
			if w.StopBlock < uint64(readAt-start) && err.Error() == "CRC mismatch in block" {
				return fmt.Errorf("CRC failed %s:%d: %w", path(locs[k]), locs[k].block, err)
			}
			return fmt.Errorf("failed to process block %s:%d: %w", path(locs[k]), locs[k].block, err)
		}
		if readErr != nil {
			// wal.go:378-380 returns with position on the unreadable block and
			// Offset as the block before it left it: CRC_SIZE (:393), or the
			// caller's Offset when it is the first block of the call.  readAt is
			// an index into locs (the whole call), not into this window, so a
			// window restarted at a pending fragment (start > 0) still gives
			// CRC_SIZE, which is what the reference's one pass holds there.
			off := uint64(crc.CRC_SIZE)
			if readAt == 0 {
				off = position.Offset
			}
			setPos(readAt, off)
			return readErr
		}
		switch {
		case hi == len(locs) || w.PendBlock < 0:
			start, offset, window = hi, crc.CRC_SIZE, recoverWindowBlocks
		case w.PendBlock == 0 && w.PendOffset == offset: // one record longer than the window
			window *= 2
		default: // rebuild the record split at the window's end from its first fragment
			start, offset, window = start+int(w.PendBlock), w.PendOffset, recoverWindowBlocks
		}
	}
	// every written block replayed: past the last log (wal.go:400-405)
	if len(locs) > 0 {
		position.Offset = crc.CRC_SIZE
	}
	position.LogIndex, position.BlockIndex = wal.lastLogIndex+1, 0
	return nil
}
