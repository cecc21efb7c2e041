/* Host platform layer: pio peripheral (replaced by the synthetic capture). */
#pragma once
