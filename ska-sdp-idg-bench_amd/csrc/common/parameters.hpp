// parameters.hpp -- compile-time constants of the benchmark.
// Same values as the reference's app/common/parameters.hpp:3-5.
#pragma once

#define NR_CORRELATIONS 4
#define IMAGE_SIZE 0.01f
#define W_STEP 0
