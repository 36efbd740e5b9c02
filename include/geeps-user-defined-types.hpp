#ifndef __geeps_user_defined_types_hpp__
#define __geeps_user_defined_types_hpp__

/*
 * This header restates the public API of GeePS (cuihenggang/geeps), whose
 * interface it must keep byte-for-byte so applications link unchanged.  The
 * upstream notice for that interface:
 *
 * Copyright (c) 2016, Carnegie Mellon University.
 * All rights reserved.
 *
 * Redistribution and use in source and binary forms, with or without
 * modification, are permitted provided that the following conditions
 * are met:
 * 1. Redistributions of source code must retain the above copyright
 *    notice, this list of conditions and the following disclaimer.
 * 2. Redistributions in binary form must reproduce the above copyright
 *    notice, this list of conditions and the following disclaimer in the
 *    documentation and/or other materials provided with the distribution.
 * 3. Neither the name of the University nor the names of its contributors
 *    may be used to endorse or promote products derived from this software
 *    without specific prior written permission.
 *
 * THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS
 * ``AS IS'' AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT
 * LIMITED TO, THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR
 * A PARTICULAR PURPOSE ARE DISCLAIMED.  IN NO EVENT SHALL THE COPYRIGHT
 * HOLDERS OR CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT,
 * INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING,
 * BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS
 * OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED
 * AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT
 * LIABILITY, OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY
 * WAY OUT OF THE USE OF THIS SOFTWARE, EVEN IF ADVISED OF THE
 * POSSIBILITY OF SUCH DAMAGE.
 */

// Row value and key types of the GeePS public API, for the MI355X libgeeps.
//
// Drop-in for the reference header of the same name
// (include/geeps-user-defined-types.hpp:41-73 in cuihenggang/geeps): every
// typedef, the ROW_DATA_SIZE constant and the ArrayData layout (128 floats,
// 512 bytes, zero-initialised by its constructor) are identical, so code
// compiled against either header links against either library.  The layout is
// checked against the reference header by tests/test_layout.py.

#include <stdint.h>

#include <limits>
#include <string>
#include <utility>
#include <vector>

typedef unsigned int uint;

typedef uint8_t command_t;
typedef size_t row_idx_t;
typedef float val_t;
typedef size_t table_id_t;
typedef int iter_t;

typedef std::pair<table_id_t, row_idx_t> TableRow;
typedef struct {
  table_id_t table;
  row_idx_t row;
} table_row_t;

// Values per row.  Fixed by the API; the device kernels take the row width as
// a runtime argument (include/gp_reduce.h).
#define ROW_DATA_SIZE 128

struct ArrayData {
  val_t data[ROW_DATA_SIZE];

  void init() {
    for (size_t i = 0; i < ROW_DATA_SIZE; i++) data[i] = 0;
  }
  ArrayData() { init(); }

  // Kept for source compatibility with apps that archive rows; only
  // instantiated by such apps.
  template <class Archive>
  void serialize(Archive &ar, const unsigned int /*version*/) {
    ar & data;
  }
};

typedef ArrayData RowData;
typedef ArrayData RowOpVal;

#endif  // __geeps_user_defined_types_hpp__
