/* Host platform layer: irq peripheral (replaced by the synthetic capture). */
#pragma once
