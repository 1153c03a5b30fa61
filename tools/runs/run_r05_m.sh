#!/bin/bash
cd "$(dirname "$0")/../.."
TAG=r05m bash tools/gpu_measure.sh x6prof=1,128,1,0,0,0,0,1,1 x6prof=1,32,0,0,0,0,0,0,2
