// build_id.cpp -- which sources this library was built from.
//
// IBWA_SRC_HASH is the first 16 hex digits of the SHA-256 of every *.cpp, *.h and *.hip file in
// ibwa_amd/csrc followed by every include/*.h (each list in byte order of the file names),
// computed by the Makefile at build time.  ibwa_amd/_native.py computes the same digest from the
// sources next to the library and refuses a library built from other sources, so a GPU run can
// never use a stale prebuilt .so without saying so.
#include "ibwa_aln.h"

#ifndef IBWA_SRC_HASH
#error "IBWA_SRC_HASH is set by the Makefile"
#endif

extern "C" const char *ibwa_build_id(void) { return IBWA_SRC_HASH; }
