/*
 * qparams.h -- the dynamic rect's forward quantiser at one QP (shared by the
 * host geometry, engine.h's DynGeom, and the device coder, dyn_device.h).
 */
#pragma once

#include <stdint.h>

/* MF of the (even, even) / (odd, odd) / mixed 4x4 positions, qbits = 15 +
 * QP / 6, rounding offset f = 2^qbits / 6 (inter) */
typedef struct {
    int32_t mf0, mf1, mf2, qbits, qf;
} QParams;
