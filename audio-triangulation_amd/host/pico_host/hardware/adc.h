/* Host platform layer: adc peripheral (replaced by the synthetic capture). */
#pragma once
