# k_crc_any: windows of at most 2^5 messages on every batch
SUBS = [("  uint32_t lgw = 6;\n", "  uint32_t lgw = 5;\n")]
