// pcm_common.hpp — helpers shared by the translation units of libpcmkm.so.
#pragma once
#include <string>

// Record the message of a failure for pcm_last_error (per calling thread) and
// return `code`.  Defined in pcm_engine.hip.
int pcm_fail(int code, const std::string &msg);
