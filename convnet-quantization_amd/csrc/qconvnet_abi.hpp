// Internal include: the public C ABI plus shared host-side helpers.
#pragma once
#include "qconvnet.h"
