// host_error.h — set spt_last_error() from the host-side readers (capi.cpp).
#pragma once
#include "../../include/spt.h"

// Formats the message into spt_last_error() and returns code.
spt_status spt_set_error(spt_status code, const char* fmt, ...);
