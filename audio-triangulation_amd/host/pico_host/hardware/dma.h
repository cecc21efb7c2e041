/* Host platform layer: dma peripheral (replaced by the synthetic capture). */
#pragma once
