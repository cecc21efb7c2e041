/* Host platform layer: timer peripheral (replaced by the synthetic capture). */
#pragma once
