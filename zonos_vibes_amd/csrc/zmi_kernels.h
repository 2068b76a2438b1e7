// Internal include: the public C ABI plus shared constants.
#pragma once
#include "zonos_hip.h"

#define ZMI_EOS 1024
#define ZMI_MASK 1025
#define ZMI_NCB 9
#define ZMI_VOCAB 1026
