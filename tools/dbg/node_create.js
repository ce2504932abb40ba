'use strict'
const path = require('path')
const addon = require(path.join(__dirname, '..', '..', 'hypermerge_amd', '_lib', 'hmgpu.node'))
try { addon.createStore(0, 8); console.log('createStore ok') } catch (e) { console.log('createStore failed: ' + e.message) }
