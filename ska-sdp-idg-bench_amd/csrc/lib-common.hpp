// lib-common.hpp -- public entry header of the common layer (types, synthetic
// data, reporting, work model).  Same role and include name as the
// reference's app/lib-common.hpp.
#pragma once

#include "common/common.hpp"
#include "common/math.hpp"
