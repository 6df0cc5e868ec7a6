// kingdb_amd/kingdb_include/algorithm/compressor.h -- the drop-in's face inside a
// KingDB source tree.
//
// Put this directory BEFORE the KingDB root on the include path
// (-I<repo>/kingdb_amd/kingdb_include -I. -I./include, see INTEGRATION.md level 2):
// every `#include "algorithm/compressor.h"` in KingDB (interface/database.h:33,
// interface/multipart.h:23, unit-tests/test_compression.cc:1) then resolves here,
// so every translation unit sees ONE definition of kdb::CompressorLZ4 -- the
// drop-in (kingdb_amd/csrc/compressor.h) -- and algorithm/compressor.cc +
// algorithm/lz4.cc leave the build (replaced by kingdb_amd/csrc/compressor.cc and
// libkdb_lz4.so).  The include guard is the reference header's own
// (algorithm/compressor.h:5), so the original can never be pulled in beside it.
#ifndef KINGDB_COMPRESSOR_H_
#define KINGDB_COMPRESSOR_H_

#ifndef KDB_LZ4_IN_KINGDB
#define KDB_LZ4_IN_KINGDB 1
#endif

// What algorithm/compressor.h:8-20 brought in transitively, minus algorithm/lz4.h
// (no KingDB file outside the codec names an LZ4_* symbol).
#include "util/debug.h"

#include <algorithm>
#include <cinttypes>
#include <map>

#include "util/logger.h"
#include "util/status.h"
#include "util/byte_array.h"
#include "thread/threadstorage.h"
#include "algorithm/crc32c.h"

#include "../../csrc/compressor.h"

#endif  // KINGDB_COMPRESSOR_H_
