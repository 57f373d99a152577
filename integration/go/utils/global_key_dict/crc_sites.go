// Row f4: the shadow CRC sites of utils/global_key_dict routed through
// libhundcrc (via the utils/crc cgo binding) instead of hash/crc32.  These
// are drop-in replacements for the method bodies at
// /root/reference/utils/global_key_dict/global_key_dict.go:394-416 and the
// two direct crc32.ChecksumIEEE calls in initializeNewFile (:365, :377).
// The dictionary keeps its own error texts ("data block too small to contain
// CRC", "CRC mismatch in data block"); only the arithmetic moves.
// Not compiled here (no Go toolchain); see INTEGRATION.md.
package global_key_dict

import (
	"encoding/binary"
	"errors"

	crc_util "hunddb/utils/crc"
)

// verifyBlockCRC (global_key_dict.go:394-408).
func (dict *GlobalKeyDict) verifyBlockCRC(data []byte) error {
	if len(data) < CRC_SIZE {
		return errors.New("data block too small to contain CRC")
	}
	if binary.LittleEndian.Uint32(data[0:CRC_SIZE]) != crc_util.GetCRC(data[CRC_SIZE:]) {
		return errors.New("CRC mismatch in data block")
	}
	return nil
}

// addCRCToData (global_key_dict.go:412-416): same in-place stamp as
// crc_util.AddCRCToBlockData.
func (dict *GlobalKeyDict) addCRCToData(data []byte) []byte {
	return crc_util.AddCRCToBlockData(data)
}

// initializeNewFile (:365, :377) then reads:
//
//	headerBlock = crc_util.AddCRCToBlockData(headerBlock)
//	dataBlock = crc_util.AddCRCToBlockData(dataBlock)
