#!/bin/sh
echo "Hello World!"
